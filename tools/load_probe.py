"""Index load at scale: build the bench's index (bench.py CONFIGS), save it
as `.idx`, load it back (sahara_gpu_open_file, the CLI's path) with
SAHARA_TIMING set (the load's steps on stderr), and check the loaded index
against the built one: the whole SA and text (export_sa / export_text) and
the hits of a read sample, all four execution modes' default.

usage: python tools/load_probe.py [--config c3] [--reads 200000] [--loads 2] [--dir /tmp]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reads", type=int, default=200000)
    ap.add_argument("--loads", type=int, default=2)
    ap.add_argument("--dir", default="/tmp")
    a = ap.parse_args()
    os.environ["SAHARA_TIMING"] = "1"
    import bench
    import sahara_amd as sa
    ref_len, nrec, _, rlen, k, edit, gen = bench.CONFIGS[a.config]
    flat, lens = sa.synth_reference(bench.record_lengths(ref_len, nrec), sigma=6, seed=42)
    t = time.time()
    built = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)
    print(f"build {time.time() - t:.2f} s", flush=True)
    reads = sa.synth_reads(flat, lens, a.reads, rlen, k if edit else 0, sigma=6, seed=7)
    del flat
    path = os.path.join(a.dir, f"load_probe_{a.config}.idx")
    t = time.time()
    built.save(path)
    print(f"save {time.time() - t:.2f} s, {os.path.getsize(path) / 1e9:.2f} GB", flush=True)
    scheme = sa.search_scheme(gen, 0, k, rlen, hamming=not edit)
    pats = sa.interleave_rc(reads, 6)
    want = sa.search(built, pats, scheme, edit=edit)
    sa_b, text_b = built.export_sa(), built.export_text()
    built.close()
    try:
        for i in range(a.loads):
            t = time.time()
            idx = sa.BiFMIndex.load(path, device=0)
            print(f"load {i}: {time.time() - t:.3f} s", flush=True)
            if i == 0:
                same_sa = np.array_equal(idx.export_sa(), sa_b)
                same_text = np.array_equal(idx.export_text(), text_b)
                got = sa.search(idx, pats, scheme, edit=edit)
                same_hits = len(got) == len(want) and np.array_equal(got, want)
                print(f"loaded == built: sa {same_sa} text {same_text} hits {same_hits} ({len(want)})", flush=True)
                if not (same_sa and same_text and same_hits):
                    sys.exit(1)
            idx.close()
    finally:
        os.remove(path)


if __name__ == "__main__":
    main()
