"""Does the thread that creates a context matter? The bench workload's packed
call (sahara_gpu_search_packed_compact) timed on a context built on the main
thread and on one built on a helper thread that has exited since, alternating.

usage: python tools/thread_probe.py [--config c3] [--rounds 2] [--steps 5]
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
    a = ap.parse_args()
    import bench
    import sahara_amd as sa
    ref_len, nrec, nreads, rlen, k, edit, gen = bench.CONFIGS[a.config]
    flat, lens = sa.synth_reference(bench.record_lengths(ref_len, nrec), sigma=6, seed=42)
    reads = sa.synth_reads(flat, lens, nreads, rlen, k if edit else 0, sigma=6, seed=7)
    scheme = sa.search_scheme(gen, 0, k, rlen, hamming=not edit)
    packed = sa.pack_reads(reads, 6, pinned=True)
    idx = {"main": sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)}
    holder = {}
    t = threading.Thread(target=lambda: holder.update(i=sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)))
    t.start()
    t.join()
    idx["helper"] = holder["i"]
    del flat
    for r in range(a.rounds):
        for name, ix in idx.items():
            for _ in range(2):
                sa.search_packed_compact(ix, packed, scheme, edit=edit).close()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                sa.search_packed_compact(ix, packed, scheme, edit=edit).close()
            el = time.perf_counter() - t0
            print(f"round {r} context built on {name:6s} thread: {nreads * a.steps / el / 1e6:8.1f}M reads/s", flush=True)


if __name__ == "__main__":
    main()
