"""Host packing speed of the library's own packer (sahara_pack_2bit) from T
Python threads over the bench's 1 GB read array, against a copy of it in
freshly first-touched memory: is the streamed upload's packing slower than
tools/probe/pack_bench because of the input's pages?"""
import ctypes as C
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import sahara_amd as sa  # noqa: E402

L = sa.lib()
lens = bench.record_lengths(300_000_000, 24)
flat, lens = sa.synth_reference(lens, sigma=6, seed=42)
t = time.time()
reads = sa.synth_reads(flat, lens, 10_000_000, 100, 2, sigma=6, seed=7)
print(f"reads synthesised in {time.time() - t:.1f}s", flush=True)
fresh = np.empty_like(reads)
fresh[:] = reads


def run(arr, T, piece=4 << 20):
    flatr = arr.reshape(-1)
    n = flatr.size
    out = np.zeros(n // 4 + 64, np.uint8)
    pieces = [(lo, min(n, lo + piece)) for lo in range(0, n, piece)]

    def work(t):
        cnt = C.c_uint64()
        for k in range(t, len(pieces), T):
            lo, hi = pieces[k]
            L.sahara_pack_2bit(flatr[lo:].ctypes.data_as(C.POINTER(C.c_uint8)), hi - lo, 6, 0,
                               out[lo // 4:].ctypes.data_as(C.POINTER(C.c_uint8)), None, 0, C.byref(cnt))
    best = 1e9
    for _ in range(3):
        th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        best = min(best, time.perf_counter() - t0)
    return n / best / 1e9, best * 1e3


for T in (1, 8, 16):
    for name, arr in (("bench reads", reads), ("fresh copy", fresh)):
        gbs, ms = run(arr, T)
        print(f"threads {T:2d} {name:12s} {gbs:6.1f} GB/s {ms:7.2f} ms per GB", flush=True)
