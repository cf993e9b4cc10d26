"""Does the thread that creates a context matter? The bench workload's packed
call (sahara_gpu_search_packed_compact) timed on a context built on the main
thread and on one built on a helper thread that has exited since, alternating.

usage: python tools/thread_probe.py [--config c3] [--rounds 2] [--steps 5] [--exited] [--alive]
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--exited", action="store_true", help="also a context built on a helper thread that has exited")
    ap.add_argument("--alive", action="store_true", help="also a helper thread that builds, searches and closes")
    ap.add_argument("--env", default="", help="VAR=VAL,... set for a second pass of every case")
    a = ap.parse_args()
    import bench
    import sahara_amd as sa
    ref_len, nrec, nreads, rlen, k, edit, gen = bench.CONFIGS[a.config]
    flat, lens = sa.synth_reference(bench.record_lengths(ref_len, nrec), sigma=6, seed=42)
    reads = sa.synth_reads(flat, lens, nreads, rlen, k if edit else 0, sigma=6, seed=7)
    scheme = sa.search_scheme(gen, 0, k, rlen, hamming=not edit)
    packed = sa.pack_reads(reads, 6, pinned=True)
    idx = {"main": sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)}
    if a.exited:  # (two resident indexes: ~180 GB of HBM at C3)
        holder = {}
        t = threading.Thread(target=lambda: holder.update(i=sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)))
        t.start()
        t.join()
        idx["helper"] = holder["i"]
    flat0 = flat
    def timed(ix):
        for _ in range(2):
            sa.search_packed_compact(ix, packed, scheme, edit=edit).close()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            sa.search_packed_compact(ix, packed, scheme, edit=edit).close()
        v = nreads * a.steps / (time.perf_counter() - t0)
        st = ix.stats()
        print(f"    ({threading.current_thread().name}: stage {st['stage_ms']:.2f} ms, text {st['text_ms']:.2f} ms, "
              f"search {st['search_ms']:.2f} ms (grid {st['search_grid']}, launches {st['search_launches']}), text grid {st['text_grid']}, locate {st['locate_ms']:.2f} ms, chunks {list(st['upload_chunks'])}, "
              f"total {st['total_ms']:.2f} ms)", flush=True)
        return v
    for r in range(a.rounds):
        for name, ix in idx.items():
            print(f"round {r} context built on {name:6s} thread: {timed(ix) / 1e6:8.1f}M reads/s", flush=True)
        if not a.alive:
            continue
        # a helper thread that builds a context and searches on it while alive
        out = {}

        def alive():
            ix = sa.BiFMIndex.build_flat(flat0, lens, sigma=6, device=0)
            out["v"] = timed(ix)
            ix.close()
        t = threading.Thread(target=alive)
        t.start()
        t.join()
        print(f"round {r} context built and searched on a live helper thread: {out['v'] / 1e6:8.1f}M reads/s", flush=True)


if __name__ == "__main__":
    main()
