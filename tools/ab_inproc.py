"""Device-resident A/B of SAHARA_* settings in one process: the bench workload
(bench.py CONFIGS) is built and staged once, then each setting's timed steps
run in alternating rounds (the library reads its variables per pass).

usage: python tools/ab_inproc.py [--config c3] [--rounds 3] [--steps 10] [--count] [--packed] NAME=VAR=VAL[,VAR=VAL] ...

--packed times the bench's headline call instead (sahara_gpu_search_packed_compact
from host reads two bits per symbol, hits into host memory).
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--count", action="store_true", help="one instrumented run per setting (lane utilisation)")
    ap.add_argument("--packed", action="store_true", help="time the packed-reads compact call (bench value)")
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    import bench
    import sahara_amd as sa
    ref_len, nrec, nreads, rlen, k, edit, gen = bench.CONFIGS[a.config]
    flat, lens = sa.synth_reference(bench.record_lengths(ref_len, nrec), sigma=6, seed=42)
    idx = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=0)
    reads = sa.synth_reads(flat, lens, nreads, rlen, k if edit else 0, sigma=6, seed=7,
                           substitutions=0 if edit else k)
    del flat
    scheme = sa.search_scheme(gen, 0, k, rlen, hamming=not edit)
    idx.stage(sa.interleave_rc(reads, 6), scheme, edit=edit)
    packed = sa.pack_reads(reads, 6, pinned=True) if a.packed else None

    def one():
        if packed is None:
            return idx.run()
        h = sa.search_packed_compact(idx, packed, scheme, edit=edit)
        n = len(h)
        h.close()
        return n
    sets = []
    for s in a.settings:
        name, _, kv = s.partition("=")
        sets.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    known = {v for _, env in sets for v in env}
    res = {n: [] for n, _ in sets}
    hits = {}
    for r in range(a.rounds):
        for name, env in sets:
            for v in known:
                os.environ.pop(v, None)
            os.environ.update(env)
            one()
            one()
            t = time.perf_counter()
            tm = 0.0
            for _ in range(a.steps):
                nh = one()
                st = idx.stats()
                tm += st["text_ms"]
            el = time.perf_counter() - t
            res[name].append(nreads * a.steps / el)
            hits.setdefault(name, nh)
            extra = ""
            if a.count and r == 0:
                idx.run(count=True)
                c = idx.stats()
                it = max(1, c['text_iterations'])
                extra = (f" lane_util {c['text_active'] / (64 * it):.3f}"
                         f" steps/read {c['text_steps'] / nreads:.1f} iters {c['text_iterations']}"
                         f" refills {c['text_refills']} cy/iter refill {c['text_cycles_refill'] / it:.0f}"
                         f" step {c['text_cycles_step'] / it:.0f} emit {c['text_cycles_emit'] / it:.0f}"
                         f" count-mode text {c['text_ms']:.2f} ms launches {c['text_launches']} grid {c['text_grid']}"
                         f" stolen/read {c['text_stolen'] / nreads:.3f}")
            print(f"round {r} {name:10s} {nreads * a.steps / el / 1e6:8.1f}M reads/s {el * 1e3 / a.steps:7.2f} ms/step "
                  f"text {tm / a.steps:6.2f} ms hits {nh}{extra}", flush=True)
    base = None
    for name, v in res.items():
        mean = float(np.mean(v))
        base = base or mean
        print(f"{name:10s} " + " ".join(f"{x / 1e6:.1f}" for x in v) + f"  mean {mean / 1e6:.1f}M ({mean / base:.3f})"
              f"  hits {hits[name]}")
    assert len(set(hits.values())) == 1, "settings disagree on the hit count"


if __name__ == "__main__":
    main()
