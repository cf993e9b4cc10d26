"""Host -> device copy rate from page-locked memory (torch), the shape of the
streamed upload's chunk DMAs: 12.8 MB and 256 MB copies on one stream, the
same split over 2 and 4 streams, and device -> host. Prints GB/s per case.

usage: python tools/probe/h2d_probe.py   (HSA_ENABLE_SDMA=0: blit kernels instead of copy engines)
"""
import time

import torch


def rate(nbytes, nstreams, reps, d2h=False):
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.fill_(1)
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    part = (nbytes + nstreams - 1) // nstreams

    def once():
        for i, s in enumerate(streams):
            lo, hi = i * part, min(nbytes, (i + 1) * part)
            with torch.cuda.stream(s):
                if d2h:
                    host[lo:hi].copy_(dev[lo:hi], non_blocking=True)
                else:
                    dev[lo:hi].copy_(host[lo:hi], non_blocking=True)
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        once()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    return nbytes * reps / el / 1e9


torch.cuda.init()
for nb in (12_800_000, 256 << 20):
    for ns in (1, 2, 4):
        print(f"H2D {nb / 1e6:7.1f} MB  streams {ns}  {rate(nb, ns, 40 if nb < 1e8 else 8):6.1f} GB/s", flush=True)
for ns in (1, 2):
    print(f"D2H  256.0 MB  streams {ns}  {rate(256 << 20, ns, 8, d2h=True):6.1f} GB/s", flush=True)
