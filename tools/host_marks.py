"""Host-side marks of device-resident steps (SAHARA_TIMING=2 on sahara_gpu_run):
where a step's wall time goes outside the kernels (pass setup, issue, finisher
waits, the end-of-pass synchronisation, the Python call around it).

usage: python tools/host_marks.py [--config c3] [--steps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import bench
    import sahara_amd as sa
    ref_len, nrec, nreads, rlen, k, edit, gen = bench.CONFIGS[a.config]
    flat, lens = sa.synth_reference(bench.record_lengths(ref_len, nrec), sigma=6, seed=42)
    idx = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)
    reads = sa.synth_reads(flat, lens, nreads, rlen, k if edit else 0, sigma=6, seed=7, substitutions=0 if edit else k)
    del flat
    idx.stage(sa.interleave_rc(reads, 6), sa.search_scheme(gen, 0, k, rlen, hamming=not edit), edit=edit)
    for _ in range(3):
        idx.run()
    t = time.perf_counter()
    for _ in range(10):
        idx.run()
        idx.stats()
    print(f"plain steps: {(time.perf_counter() - t) * 100:.3f} ms/step", flush=True)
    os.environ["SAHARA_TIMING"] = "2"
    for i in range(a.steps):
        t = time.perf_counter()
        idx.run()
        t1 = time.perf_counter()
        idx.stats()
        t2 = time.perf_counter()
        print(f"step {i}: run {(t1 - t) * 1e3:.3f} ms, stats {(t2 - t1) * 1e3:.3f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
