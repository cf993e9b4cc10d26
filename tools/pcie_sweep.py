"""PCIe-inclusive path (sahara_gpu_search_reads_compact) at C3 under several
knob settings in one process (the library reads its SAHARA_* variables per
pass), alternating rounds: reads/s per setting.

usage: python tools/pcie_sweep.py [--rounds 2] [--steps 10] [--reads N] NAME=VAR=VAL[,VAR=VAL...] ...
  e.g. base= b2M=SAHARA_BATCH=2097152 ramp=SAHARA_RAMP=2
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def cgroup_stat():
    """cgroup v2 cpu.stat of this process's cgroup (throttling under a CPU quota), or {}."""
    try:
        rel = open("/proc/self/cgroup").read().strip().split("::")[-1]
        base = "/sys/fs/cgroup" + rel
        d = {}
        for line in open(os.path.join(base, "cpu.stat")):
            k, v = line.split()
            d[k] = int(v)
        try:
            d["cpu.max"] = open(os.path.join(base, "cpu.max")).read().strip()
        except OSError:
            pass
        return d
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--full", action="store_true", help="whole 24-B records (sahara_gpu_search_reads)")
    ap.add_argument("--max-hits", type=int, default=0, help="sahara_gpu_search_reads with --max_hits N")
    ap.add_argument("--read-errors", type=int, default=2, help="errors simulated per read (search k stays 2)")
    ap.add_argument("--marks", type=int, default=0, help="then this many calls with SAHARA_TIMING=2 (host marks, stderr)")
    ap.add_argument("--config", default=None, help="a bench.py config (c2, c3, c5): its text, reads and scheme")
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    import bench
    import sahara_amd as sa
    ref_len, nrec, nreads, rlen, k, edit, gen = bench.CONFIGS[a.config or "c3"]
    if a.config:
        a.reads, a.read_errors = nreads, k
    lens = bench.record_lengths(ref_len, nrec)
    flat, lens = sa.synth_reference(lens, sigma=6, seed=42)
    idx = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)
    reads = sa.synth_reads(flat, lens, a.reads, rlen, a.read_errors, sigma=6, seed=7)
    del flat
    sch = sa.search_scheme(gen, 0, k, rlen, hamming=not edit)
    aff = sorted(os.sched_getaffinity(0))
    print(f"placement {idx.placement()}, process CPUs {len(aff)} ({aff[:4]}..{aff[-4:]})", flush=True)
    cg0 = cgroup_stat()
    print(f"cgroup cpu.max {cg0.get('cpu.max')}, stat {cg0}", flush=True)
    call = ((lambda: sa.search_reads(idx, reads, sch, edit=edit)) if a.full
            else (lambda: sa.search_reads_compact(idx, reads, sch, edit=edit)))
    if a.max_hits:
        call = lambda: sa.search_reads(idx, reads, sch, edit=edit, max_hits=a.max_hits)
    sets = []
    for s in a.settings:
        name, _, kv = s.partition("=")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        sets.append((name, env))
    known = {k for _, env in sets for k in env}
    res = {n: [] for n, _ in sets}
    for r in range(a.rounds):
        for name, env in sets:
            for k in known:
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(2):
                h = call()
                del h
            cg = cgroup_stat()
            ct = os.times()
            t = time.perf_counter()
            st = {"stage_ms": 0.0}
            h = None
            for _ in range(a.steps):
                h = None
                h = call()
                st["stage_ms"] += idx.stats()["stage_ms"]
            el = time.perf_counter() - t
            ct1 = os.times()
            cg1 = cgroup_stat()
            cpu_ms = ((ct1.user - ct.user) + (ct1.system - ct.system)) * 1e3 / a.steps
            thr = {k: cg1.get(k, 0) - cg.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec")}
            n = len(h)
            del h
            rps = a.reads * a.steps / el
            res[name].append(rps)
            print(f"round {r} {name:12s} {rps/1e6:7.1f}M reads/s  {el*1e3/a.steps:6.2f} ms/call  "
                  f"packing {st['stage_ms']/a.steps:5.2f} ms  cpu {cpu_ms:6.1f} ms/call  cgroup {thr}  hits {n}", flush=True)
    for name, v in res.items():
        print(f"{name:12s} " + " ".join(f"{x/1e6:.1f}" for x in v) + f"  mean {np.mean(v)/1e6:.1f}M")
    if a.marks:
        for k in known:
            os.environ.pop(k, None)
        os.environ.update(sets[0][1])
        os.environ["SAHARA_TIMING"] = "2"
        for _ in range(a.marks):
            h = call()
            del h


if __name__ == "__main__":
    main()
