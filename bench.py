#!/usr/bin/env python3
"""bench.py — reads/s of sahara's search hot path on MI355X (BASELINE.json metric).

A "step" is one call of the hot path at the drop-in boundary, SURVEY §8(d)'s
search wall time: the workload's synthetic reads, in host memory in the form
`sahara search`'s FASTA ingest produces (two bits per symbol, N positions
listed: sahara_read_fasta form 2), go through sahara_gpu_search_packed_compact
— upload, reverse-complement interleave (search.cpp:121-123), search-scheme
DFS, locate, canonical sort — until every located hit is in host memory.
`value` = reads / that time. The same pass with the reads already resident in
HBM and the hits left there is reported as config.device_resident. Default
workload = BASELINE.json configs[2] (C3): k=2 Levenshtein, 10M x 100 bp reads
vs a 3 Gbp, 24-record synthetic reference (record lengths proportional to
GRCh38 chromosomes), default generator h2-k2. The ingest that
the timed region starts after (FASTA -> 2-bit) is timed beside it, with the
rank form it replaces (config.ingest).

Multi-GPU (torchrun, one process per GPU): every rank builds the full index
on its own GPU (replicated, as SURVEY §8(e) prescribes), searches its own
shard of 10M reads (weak scaling); the max step time and hit counts are
reduced over RCCL. No collective sits on the data path. After the timed
steps, the hit records are gathered to rank 0 over RCCL (xGMI) in a step of
their own, reported as config.hit_gather (not part of `value`).

Rank 0 at N=1 also times the CPU restatement (oracle/, the reference's
algorithm restated in C++) on a bounded sample of the same reads on the host
cores, and checks GPU == CPU hits on that sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GRCH38 = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
          138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
          83257441, 80373285, 58617616, 64444167, 46709983, 50818468, 156040895, 57227415]

CONFIGS = {
    # name: (ref_len, n_records, reads per GPU, read_len, errors, edit, generator)
    "c1": (1_000_000, 1, 1_000, 32, 0, True, "h2-k2"),
    "c2": (100_000_000, 1, 1_000_000, 100, 1, False, "h2-k2"),
    "c3": (3_000_000_000, 24, 10_000_000, 100, 2, True, "h2-k2"),
    "c5": (3_000_000_000, 24, 1_000_000, 250, 3, True, "h2-k2"),
    # beyond BASELINE: a 6 Gbp text (two GRCh38-shaped haplotypes) exceeds
    # 32-bit rows and is indexed in two parts
    "c6": (6_000_000_000, 48, 10_000_000, 100, 2, True, "h2-k2"),
}

METRIC = "reads/s at k=2 edit, 10M×100bp vs 3Gbp index; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# wave64 VALU instructions per second: 256 CUs x 4 SIMDs x 2.4 GHz, one
# instruction per SIMD every 2 cycles (MI355X_MICROARCH.md: 32 lanes/cycle)
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2
# sahara_hit (include/sahara_hip.h) as numpy: the fields hits_digest reads
HIT_DTYPE_BENCH = np.dtype([("qid", "<u8"), ("seq_id", "<u4"), ("err", "<u4"), ("pos", "<u8")])


def log(*a):
    print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def record_lengths(total, n):
    if n == 1:
        return np.array([total], np.uint64)
    w = np.resize(np.array(GRCH38, np.float64), n)
    lens = np.floor(w / w.sum() * total).astype(np.uint64)
    lens[0] += np.uint64(total - int(lens.sum()))
    return lens


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    # the GPU box grants 16 host cores per GPU (OMP_NUM_THREADS is set to it)
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return max(1, min(n, 16))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--reads", type=int, default=0, help="override reads per GPU")
    ap.add_argument("--ref-len", type=int, default=0, help="override reference length")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the instrumented (untimed) counter run")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the secondary PCIe-inclusive calls (rank reads, whole records, host patterns)")
    ap.add_argument("--no-ingest", action="store_true", help="skip timing the FASTA ingest (both forms)")
    ap.add_argument("--no-device-resident", action="store_true",
                    help="skip the device-resident pass (profiling: every search launch then has the timed call's "
                         "shape); implies --no-count --no-verify --no-e2e --no-ref-path --no-cpu")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the timed RCCL gather of hit records")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the full-size checks (origin recall; GPU suffix array against the text)")
    ap.add_argument("--no-ref-path", action="store_true",
                    help="skip the timed reference-execution pass (FM ranks from the root + LF locate)")
    ap.add_argument("--execution", default="default", choices=["default", "reference"],
                    help="reference: the timed steps run the reference's execution model (profiling its kernels)")
    ap.add_argument("--traffic-json", default=None,
                    help="measured HBM bytes per launch per kernel (tools/traffic.sh + tools/traffic_summary.py); "
                         "default profiles/traffic_<config>.json when it exists")
    args = ap.parse_args()

    if args.no_device_resident:
        if args.execution == "reference":
            ap.error("--execution reference times the device-resident pass: it cannot go with --no-device-resident")
        args.no_count = args.no_verify = args.no_e2e = args.no_ref_path = args.no_cpu = True
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # six streams per context (seeds, FM, text, locate, upload, download): give
    # them their own hardware queues (HIP's default is 4 per process; measured
    # 235M -> 252M reads/s on the PCIe-inclusive path at C3)
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    import torch  # plumbing only: device sync + torch.distributed (RCCL)
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import sahara_amd as sa

    ref_len, nrec, nreads, rlen, k, edit, gen = CONFIGS[args.config]
    if args.ref_len:
        ref_len = args.ref_len
    if args.reads:
        nreads = args.reads
    sigma = 6

    lens = record_lengths(ref_len, nrec)
    t = time.time()
    flat, lens = sa.synth_reference(lens, sigma=sigma, seed=42)
    log(f"rank {rank}: reference {ref_len/1e9:.3f} Gbp in {len(lens)} records ({time.time()-t:.1f}s)")
    t = time.time()
    idx = sa.BiFMIndex.build_flat(flat, lens, sigma=sigma, sampling_rate=16, device=local)
    build_s = time.time() - t
    info = idx.info()
    log(f"rank {rank}: GPU index built in {build_s:.1f}s, {info['device_bytes']/1e9:.2f} GB resident")

    t = time.time()
    # exactly k errors per read, of uniform type S/I/D for edit
    # distance and substitutions for Hamming (C2)
    reads, origin = sa.synth_reads(flat, lens, nreads, rlen, k if edit else 0, sigma=sigma, seed=7 + 1000003 * rank,
                                   substitutions=0 if edit else k, with_origin=True)
    pats = sa.interleave_rc(reads, sigma)
    scheme = sa.search_scheme(gen, 0, k, rlen, hamming=not edit)
    log(f"rank {rank}: {nreads} reads simulated ({time.time()-t:.1f}s), {scheme[0].shape[0]} searches")
    # the timed call's input: the reads as `sahara search`'s FASTA ingest hands
    # them over — two bits per symbol in page-locked memory, N positions
    # listed (sahara_read_fasta form 2) — from the reads written as a FASTA
    # file and read back, the ingest timed in both forms (--no-ingest: the
    # library's packer fills the same form)
    ingest = None
    if not args.no_ingest:
        ingest, packed = time_ingest(sa, reads, sigma)
    else:
        packed = sa.pack_reads(reads, sigma, pinned=True)
    if args.execution == "reference":  # profiling aid: the timed steps are the reference's execution model
        args.no_count = args.no_ref_path = True

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- the headline: SURVEY §8(d)'s search wall time per call, host reads
    # (packed) in, every located hit in host memory out
    # (a multi-part index, C6: whole 24-B records, sahara_gpu_search_packed;
    # compact records address one part's text)
    multi_part = info["n_parts"] > 1

    class _Whole:  # the whole-records call's result with CompactHits' surface
        def __init__(self, hits):
            self.hits = hits

        def close(self):
            pass

        def __len__(self):
            return len(self.hits)

        def to_hits(self):
            return self.hits

    if multi_part:
        packed_call = lambda: _Whole(sa.search_packed(idx, packed, scheme, edit=edit))  # noqa: E731
    else:
        packed_call = lambda: sa.search_packed_compact(idx, packed, scheme, edit=edit)  # noqa: E731
    step_stats = {"search_ms": 0.0, "text_ms": 0.0, "locate_ms": 0.0, "sort_ms": 0.0, "seed_ms": 0.0,
                  "stage_ms": 0.0, "output_ms": 0.0, "search_launches": 0, "text_launches": 0}
    h = None
    last_result = None
    if args.execution != "reference":
        # two warmup calls whatever --warmup says: the first sizes the hit
        # sink from its own result, the second pins it into the pool every
        # later call draws from (capi.cpp allocPinned)
        for i in range(max(2, args.warmup)):
            t = time.time()
            h = packed_call()
            h.close()
            log(f"rank {rank}: warmup {i} {time.time()-t:.3f}s")
        h = None
        barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            if h is not None:
                h.close()  # the previous call's records back to the pool (sahara_gpu_free_blocks)
            h = packed_call()
            st = idx.stats()
            for kk in step_stats:
                step_stats[kk] += st[kk]
        barrier()
        elapsed = time.perf_counter() - t0
        n_packed = len(h)
        packed_hits = h.to_hits()
        last_result = h  # gathered to rank 0 after the timing (N > 1), then closed

    # ---- the same pass device-resident: reads staged in HBM, hits left there
    dr_stats = {"search_ms": 0.0, "text_ms": 0.0, "search_launches": 0, "text_launches": 0}
    if args.no_device_resident:
        dr_elapsed, nh, digest = None, n_packed, None
    else:
        idx.stage(pats, scheme, edit=edit)
        if args.execution == "reference":
            idx.set_mode(verify=False, locate_sa=False)
        for i in range(args.warmup):
            idx.run()
        barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            nh = idx.run()
            st = idx.stats()
            for kk in dr_stats:
                dr_stats[kk] += st[kk]
        barrier()
        dr_elapsed = time.perf_counter() - t0
        digest = idx.digest()
    if args.execution == "reference":  # the timed steps are this mode's
        elapsed, step_stats, n_packed, packed_hits = dr_elapsed, dr_stats, nh, None

    gather = None
    per_rank = None
    if world > 1:
        from sahara_amd.dist import max_over_ranks, sum_over_ranks, values_of_ranks
        per_rank = {"index_build_s": [round(v, 2) for v in values_of_ranks(build_s, device="cuda")],
                    "ms_per_step": [round(v * 1e3 / args.steps, 3) for v in values_of_ranks(elapsed, device="cuda")],
                    "device_resident_ms_per_step": [round(v * 1e3 / args.steps, 3)
                                                    for v in values_of_ranks(dr_elapsed or 0.0, device="cuda")],
                    "hits": [int(v) for v in values_of_ranks(nh, device="cuda")]}
        elapsed = max_over_ranks(elapsed, device="cuda")  # RCCL over xGMI
        dr_elapsed = max_over_ranks(dr_elapsed, device="cuda") if dr_elapsed else None
        total_hits = sum_over_ranks(nh, device="cuda")
        if not args.no_gather and last_result is not None:
            gather = gather_step(last_result, getattr(last_result, "rec_starts", None), nreads, world, rank, barrier,
                                 dist, torch)
    else:
        total_hits = nh
    if last_result is not None:
        last_result.close()
        last_result = None
    same_hits = None if digest is None else (n_packed == nh and (packed_hits is None or
                                                                  hits_digest(packed_hits) == digest))

    # full-size checks that do not lean on the GPU's own index: every read is
    # found where it was sampled (all ranks), and rank 0 checks the whole GPU
    # suffix array, BWT and samples against the synthetic text with torch ops
    checks = {}
    if not args.no_verify:
        t = time.time()
        checks["origin_recall"] = origin_recall(idx.fetch(), origin, k)
        if world > 1:
            from sahara_amd.dist import values_of_ranks
            checks["origin_recall"] = min(values_of_ranks(checks["origin_recall"], device="cuda"))
        if rank == 0:
            checks.update(verify_index(idx, flat, lens, torch, f"cuda:{local}"))
        log(f"rank {rank}: full-size checks {checks} ({time.time()-t:.1f}s)")

    ms_per_step = elapsed * 1000.0 / args.steps
    reads_per_s = nreads * world * args.steps / elapsed
    search_ms = step_stats["search_ms"]
    text_ms = step_stats["text_ms"]
    launches = step_stats["search_launches"]
    text_launches = step_stats["text_launches"]

    # instrumented run (untimed): deterministic work counters -> algorithmic bytes
    cnt = ref_cnt = None
    if not args.no_count:
        idx.run(count=True)
        cnt = idx.stats()
        # SURVEY §8(d) B_read: the reference algorithm's bytes per read, counted
        # in the reference-execution mode (every node ranked from the root, LF
        # locate to the rate-16 samples), whose counters equal the CPU
        # restatement's (tests/test_gpu_parity.py::test_no_hits_and_device_resident_path)
        idx.set_mode(verify=False, locate_sa=False)
        idx.run(count=True)
        ref_cnt = idx.stats()
        idx.set_mode(verify=True, locate_sa=True)
    search_ms_step = search_ms / args.steps
    roofline = None
    extra = {}
    if cnt:
        # algorithmic bytes per step: FM = 64-B Occ lines touched
        # + pattern bytes; text = per task its window, task record and SA
        # entry, plus each pattern once; locate = one SA read per FM-located
        # row (the FM kernel reads each pattern as 4-bit words: patWords u32
        # per pattern, not one byte per symbol)
        search_bytes = 64.0 * cnt["ext_lines"] + pats.shape[0] * ((rlen + 7) // 8) * 4.0
        # per text task: the source blocks of its window (16-B blocks of 32
        # symbols, 3 bit planes: pass.cpp winBlocks, plus the block its
        # funnel-shifted copy starts in), the task record, and the SA entry
        # unless the task came with its text position (k-mer seeds with one
        # occurrence: text_pos_tasks); per pattern its blocks once (the tasks
        # of one pattern share them in L2)
        win_blocks = (rlen + 2 * k + 62) // 32
        pat_blocks = (rlen + 31) // 32
        text_bytes = (cnt["conversions"] * (16.0 * win_blocks + 16) + 4.0 * (cnt["conversions"] - cnt["text_pos_tasks"])
                      + pats.shape[0] * 16.0 * pat_blocks)
        locate_bytes = 4.0 * cnt["hits"]
        text_ms_step = text_ms / args.steps
        kern = {"kSearchFM": {"ms": round(search_ms_step, 2), "bytes": search_bytes,
                              "GBs": round(search_bytes / (search_ms_step / 1e3) / 1e9, 1)},
                "kSearchTextBatch": {"ms": round(text_ms_step, 2), "bytes": text_bytes,
                                "GBs": round(text_bytes / max(text_ms_step, 1e-6) * 1e3 / 1e9, 1)}}
        dom = max(kern, key=lambda n: kern[n]["ms"])
        # launches per step of the dominant kernel (the first batch's text
        # phase runs as two launches: its seed tasks, then the FM phase's)
        per_launch = max(1, (launches if dom == "kSearchFM" else text_launches) // args.steps)
        reads_per_launch = nreads / per_launch
        launch_ms = kern[dom]["ms"] / per_launch
        # The roofline prices the dominant kernel's own algorithmic bytes (what
        # it must read: DESIGN.md §3) over its launch time. SURVEY §8(d)'s
        # B_read — the bytes per read of the reference's algorithm: 64 B per
        # Occ line its DFS ranks and per located row (LF steps + the SA-sample
        # line), plus the 2L query bytes — is reported beside it: this path
        # does not move those bytes (k-mer table, text phase, full SA), so as
        # an achieved rate it is an equivalent, not a fraction of peak.
        achieved = kern[dom]["GBs"]
        b_read = (64.0 * (ref_cnt["ext_lines"] + ref_cnt["lf_steps"] + ref_cnt["hits"]) + pats.size) / nreads
        roofline = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "algorithmic_bytes_per_launch": round(kern[dom]["bytes"] / per_launch),
                    "units_per_launch": round(reads_per_launch), "launch_ms": round(launch_ms, 3),
                    "note": ("kSearchTextBatch is VALU/LDS-issue bound (DESIGN.md §3.4): its HBM fraction is small by "
                             "construction") if dom == "kSearchTextBatch" else "memory-latency bound (DESIGN.md §3.2)",
                    "survey_8d": {"B_read": round(b_read, 1),
                                  "reference_equivalent_GBs": round(b_read * reads_per_s / 1e9, 1),
                                  "reference_equivalent_frac": round(b_read * reads_per_s / 1e9 / HBM_PEAK_GBS, 3),
                                  "basis": "the reference algorithm's Occ / LF / SA-sample lines + query bytes per "
                                           "read, counted in the reference-execution mode, x reads/s"}}
        # Committed profiles carry the build id of the library they measured
        # (tools/build_id.py); one of another build is reported as stale and
        # nothing is priced on it.
        build = sa.build_id()
        tj = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(tj):
            tall = json.load(open(tj))
            tr = tall.get(dom)
            if tr and tall.get("build_id") != build:
                roofline["stale_traffic_profile"] = {"source": os.path.relpath(tj, ROOT),
                                                     "build_id": tall.get("build_id"), "this_build": build}
            elif tr:  # HBM bytes per launch from the committed PMC pass (FETCH_SIZE, calibrated)
                roofline["traffic"] = tr["bytes_per_launch"]
                roofline["traffic_GBs"] = tr["traffic_GBs"]
                roofline["traffic_source"] = os.path.relpath(tj, ROOT)
                if tr.get("avg_launch_us"):
                    # the same kernel's average launch in that committed kernel
                    # trace of this build (the traced run is slower: tracing
                    # serialises the streamed call's launches), and the fraction
                    # priced on it
                    traced_ms = tr["avg_launch_us"] / 1e3
                    roofline["traced"] = {
                        "launch_ms": round(traced_ms, 3),
                        "untraced_over_traced_same_build": round(launch_ms / traced_ms, 3),
                        "achieved": round(kern[dom]["bytes"] / per_launch / (traced_ms / 1e3) / 1e9, 1),
                        "frac": round(kern[dom]["bytes"] / per_launch / (traced_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                        "source": os.path.relpath(tj, ROOT), "build_id": build}
        # the bound that applies to kSearchTextBatch: VALU issue. Its instruction
        # count per launch comes from the committed SQ counter pass of the
        # same build and workload (tools/pmc_text.sh -> profiles/pmc_<config>.json)
        pj = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(pj):
            pall = json.load(open(pj))
            pm = pall.get(dom)
            if pm and pall.get("build_id") != build:
                roofline["stale_pmc_profile"] = {"source": os.path.relpath(pj, ROOT),
                                                 "build_id": pall.get("build_id"), "this_build": build}
            elif pm and pm.get("SQ_INSTS_VALU"):
                roofline["valu_issue"] = {
                    "valu_per_launch": pm["SQ_INSTS_VALU"],
                    "frac": round(pm["SQ_INSTS_VALU"] / (launch_ms / 1e3) / VALU_ISSUE_PEAK, 3),
                    "peak_per_s": VALU_ISSUE_PEAK,
                    "basis": "wave64 VALU instructions per launch / (launch time x 256 CU x 4 SIMD x 2.4 GHz / 2 "
                             "cycles per instruction)",
                    **{kk: pm[kk] for kk in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "issue_active", "wait_any",
                                             "valu_active", "lds_conflict", "dispatches") if kk in pm},
                    "source": os.path.relpath(pj, ROOT), "build_id": build}
                if roofline.get("traced"):  # priced on the committed trace's launch time instead
                    roofline["valu_issue"]["frac_traced"] = round(
                        pm["SQ_INSTS_VALU"] / (roofline["traced"]["launch_ms"] / 1e3) / VALU_ISSUE_PEAK, 3)
        extra = {"bytes_per_read": round((search_bytes + text_bytes + locate_bytes) / nreads, 1),
                 "kernels": {n: {"ms": v["ms"], "algorithmic_GBs": v["GBs"],
                                 "bytes_per_read": round(v["bytes"] / nreads, 1)} for n, v in kern.items()},
                 "nodes_per_read": round(cnt["nodes"] / nreads, 1),
                 "ext_lines_per_read": round(cnt["ext_lines"] / nreads, 1),
                 "rank_nodes_per_read": round(cnt["rank_nodes"] / nreads, 1),
                 "text_nodes_per_read": round(cnt["text_nodes"] / nreads, 1),
                 "conversions_per_read": round(cnt["conversions"] / nreads, 2),
                 "positioned_tasks_per_read": round(cnt["text_pos_tasks"] / nreads, 2),
                 "fm_lane_util": round(cnt["nodes"] / max(1, 64 * cnt["fm_iterations"]), 3),
                 "text_lane_util": round(cnt["text_active"] / max(1, 64 * cnt["text_iterations"]), 3),
                 "text_iterations_per_wave": round(cnt["text_iterations"] / max(1, 4 * cnt["search_grid"]), 1),
                 "text_refill_frac": round(cnt["text_refills"] / max(1, cnt["text_iterations"]), 3),
                 "text_cycle_split": {k: round(cnt[f"text_cycles_{k}"] / max(1, cnt["text_cycles_refill"]
                                                  + cnt["text_cycles_step"] + cnt["text_cycles_emit"]), 3)
                                      for k in ("refill", "step", "emit")},
                 "text_compare_steps_per_read": round(cnt["text_compare_steps"] / nreads, 1),
                 "text_steps_per_read": round(cnt["text_steps"] / nreads, 1),
                 "cursors": cnt["cursors"], "hits_per_read": round(cnt["hits"] / nreads, 3),
                 "search_ms": round(search_ms_step, 2), "text_ms": round(text_ms / args.steps, 2),
                 "locate_ms": round(step_stats["locate_ms"] / args.steps, 2),
                 "sort_ms": round(step_stats["sort_ms"] / args.steps, 2),
                 "seed_ms": round(step_stats["seed_ms"] / args.steps, 2),
                 "search_launches_per_step": launches // args.steps,
                 "text_launches_per_step": text_launches // args.steps,
                 "search_grid": cnt["search_grid"], "text_grid": cnt["text_grid"],
                 "pipelined": bool(cnt["pipelined"]),
                 "reference_algorithm": {"ext_lines_per_read": round(ref_cnt["ext_lines"] / nreads, 1),
                                         "lf_steps_per_read": round(ref_cnt["lf_steps"] / nreads, 2),
                                         "rows_per_read": round(ref_cnt["hits"] / nreads, 3),
                                         "nodes_per_read": round(ref_cnt["nodes"] / nreads, 1),
                                         "fm_lane_util": round(ref_cnt["nodes"] / max(1, 64 * ref_cnt["fm_iterations"]), 3),
                                         "same_hits": ref_cnt["hits"] == cnt["hits"]},
                 }

    extra["timed_call"] = ("sahara_gpu_search_packed_compact from host reads two bits per symbol (N listed; the "
                           "form sahara_read_fasta form 2 produces, in page-locked memory): each chunk DMAed straight "
                           "from the caller's buffer, RC interleave and pattern packing on the device (kPackFrom2), "
                           "search, locate, sort, each batch's hits as 8-B records (qid, text position, e; "
                           "sahara_hit_blocks) copied into pinned host memory recycled through sahara_gpu_free_blocks")
    if multi_part:
        extra["timed_call"] = extra["timed_call"].replace("sahara_gpu_search_packed_compact", "sahara_gpu_search_packed")
        extra["timed_call"] += "; multi-part index: whole 24-B hit records (compact records address one part)"
    # the timed calls' own launches, timed with HIP events on their streams
    # (comparable with a rocprofv3 kernel trace of this same command)
    extra["timed_launches"] = {
        "kSearchTextBatch": {"launches_per_step": text_launches / args.steps,
                        "avg_launch_ms": round(text_ms / max(1, text_launches), 4)},
        "kSearchFM": {"launches_per_step": launches / args.steps,
                      "avg_launch_ms": round(search_ms / max(1, launches), 4)}}
    extra["same_hits"] = same_hits
    if dr_elapsed:
        extra["device_resident"] = {
            "reads_per_s": round(nreads * world * args.steps / dr_elapsed, 1),
            "ms_per_step": round(dr_elapsed * 1e3 / args.steps, 2),
            "text_ms": round(dr_stats["text_ms"] / args.steps, 2),
            "text_launches_per_step": dr_stats["text_launches"] // args.steps,
            "timed_over": "sahara_gpu_run: reads (+RC) staged in HBM before timing, hits left in HBM"}
        extra["device_resident"]["timed_call_over_device_resident"] = round(
            reads_per_s / extra["device_resident"]["reads_per_s"], 3)
    if ingest:
        extra["ingest"] = ingest
    # other PCIe-inclusive calls (SURVEY §8(d)'s search wall time, as `value`):
    # host reads one rank per byte (packed on the host's threads inside the
    # call), whole 24-B records, host-interleaved patterns; timed like
    # `value`: warmup calls, then --steps calls, each handing its hit buffer
    # back before the next
    if not args.no_e2e:
        # two warmup calls whatever --warmup says: the first sizes the hit
        # buffer from its own result, the second pins it into the pool that
        # every later call draws from (capi.cpp allocHits)
        w2 = 2
        # the reads cross PCIe, reverse complements interleaved on the device,
        # the hits come back as 8-B records (sahara_gpu_search_reads_compact:
        # what `sahara search` calls; single-part indexes)
        if idx.info()["n_parts"] == 1:
            extra["pcie_inclusive_rank_reads"] = pcie_inclusive(
                lambda: sa.search_reads_compact(idx, reads, scheme, edit=edit), idx, nreads, args.steps, w2, world,
                barrier, nh, digest,
                "sahara_gpu_search_reads_compact from host reads one rank per byte: packed to two bits per symbol "
                "(N listed) on the host's threads inside the call, then as `value`")
        # the same with whole 24-B sahara_hit records (sahara_gpu_search_reads)
        extra["pcie_inclusive_full_records"] = pcie_inclusive(
            lambda: sa.search_reads(idx, reads, scheme, edit=edit), idx, nreads, args.steps, w2, world, barrier, nh,
            digest,
            "sahara_gpu_search_reads from host reads: streamed upload (four symbols per byte, N listed) + device RC interleave, "
            "search, locate, sort, hits D2H batch by batch into pinned host memory recycled through sahara_gpu_free")
        # the interleaved patterns cross PCIe (the reference's queries vector, sahara_gpu_search)
        extra["pcie_inclusive_patterns"] = pcie_inclusive(
            lambda: sa.search(idx, pats, scheme, edit=edit), idx, nreads, args.steps, w2, world, barrier, nh,
            digest,
            "sahara_gpu_search from host patterns (reads + RC interleaved on the host): streamed upload, search, "
            "locate, sort, hits D2H batch by batch into pinned host memory")
    # the reference's execution model timed on the same reads (north_star's
    # kernels: the FM DFS ranking every node from the root, LF walks to the
    # rate-16 samples); its roofline is SURVEY §8(d)'s B_read
    if not args.no_ref_path and ref_cnt:
        extra["reference_path"] = reference_path(idx, ref_cnt, nreads, pats.size, min(args.steps, 3), world,
                                                 barrier, args.config)
    extra.update(checks)
    if per_rank:
        extra["per_rank"] = per_rank

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(sa, idx, pats, scheme, edit, nreads, args.cpu_seconds, packed_hits)
    packed_hits = None

    out = {
        "metric": METRIC,
        "value": round(reads_per_s, 1),
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": f"{args.config.upper()}: k={k} {'lev' if edit else 'ham'}, {nreads}x{rlen}bp reads "
                               f"(+RC) per GPU vs {ref_len/1e9:g} Gbp {len(lens)}-record index, {gen}",
                   "reads_per_gpu": nreads, "read_len": rlen, "errors": k, "ref_len": ref_len,
                   "records": int(len(lens)), "generator": gen, "searches": int(scheme[0].shape[0]),
                   "parallelism": f"replicated-index x{world} (query shards)", "index_build_s": round(build_s, 1),
                   "hits_total": total_hits, "build_id": sa.build_id(), **extra},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if gather:
        gather["reads_per_s_incl_gather"] = round(nreads * world / (ms_per_step / 1e3 + gather["ms"] / 1e3), 1)
        out["config"]["hit_gather"] = gather
    if cpu and cpu.get("value"):
        out["config"]["gpu_over_cpu"] = round(reads_per_s / cpu["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def time_ingest(sa, reads, sigma):
    """The FASTA ingest that the timed region starts after, timed in both
    forms on the same reads written as a FASTA file (80 columns, one header
    per read, in /dev/shm when there is one): FASTA -> one rank per byte (the
    reference's form, search.cpp:111-130) and FASTA -> two bits per symbol +
    N list in page-locked memory (what `sahara search` hands to
    sahara_gpu_search_packed_compact), on the host threads the CLI uses.
    Returns the timings and the 2-bit form as PackedReads (checked against
    the library's packer over the reads)."""
    import tempfile
    d = "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None
    n, m = reads.shape
    chars = np.frombuffer(b"$ACGNT" if sigma == 6 else b"$ACGT", np.uint8)
    t = time.time()
    # ">%09d" header lines, then the read in 80-column lines
    head = np.empty((n, 11), np.uint8)
    head[:, 0] = ord(">")
    head[:, 10] = ord("\n")
    ids = np.arange(n, dtype=np.int64)
    for dgt in range(9):
        head[:, 9 - dgt] = 48 + (ids // 10 ** dgt) % 10
    lines = [(j, min(m, j + 80)) for j in range(0, m, 80)]
    body = np.empty((n, m + len(lines)), np.uint8)
    o = 0
    for a, b in lines:
        body[:, o:o + b - a] = chars[reads[:, a:b]]
        body[:, o + b - a] = ord("\n")
        o += b - a + 1
    fd, path = tempfile.mkstemp(suffix=".fa", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(np.concatenate([head, body], axis=1).tobytes())
        size = os.path.getsize(path)
        write_s = time.time() - t
        threads = host_threads()
        out = {"fasta_bytes": size, "threads": threads, "file": "tmpfs" if d else "tmp"}
        for form, name in ((1, "ranks"), (2, "two_bit")):
            best = None
            for _ in range(2):  # the second read is warm in the page cache
                r = None
                t = time.perf_counter()
                r = sa.read_fasta(path, sigma, form=form, threads=threads)
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            out[f"{name}_s"] = round(best, 3)
            out[f"{name}_reads_per_s"] = round(n / best, 1)
        codes, pos, _ = sa.pack_2bit(reads, sigma)
        out["two_bit_equals_packer"] = bool(np.array_equal(r["data"], codes) and
                                            np.array_equal(r["n_pos"], pos.astype(np.uint64)))
        del codes, pos
        log(f"ingest: {size/1e9:.2f} GB FASTA (written in {write_s:.1f}s): ranks {out['ranks_s']}s, "
            f"2-bit {out['two_bit_s']}s on {threads} threads")
        return out, sa.PackedReads(r["data"], n, m, r["n_pos"])
    finally:
        os.unlink(path)


def gather_step(result, rec_starts, nreads, world, rank, barrier, dist, torch, device="cuda"):
    """the last timed call's hits gathered to rank 0 over
    RCCL (xGMI). The records are the ones sahara_gpu_search_packed_compact
    left in this rank's host memory — 8-B compact records and their block
    table (first qid and end of each batch) — which go host -> device, are
    gathered to rank 0 (sahara_amd.dist.gather_compact_records) and come back
    to its host memory there, with global qids (the rank's first pattern
    added to its block qids). A whole-records result (multi-part index) is
    gathered as (qid, seq_id, pos, e) rows instead. Timed on its own (barrier
    + synchronize on both sides, max over ranks) and reported beside `value`
    (config.hit_gather, with the rate including it); verified after the timing
    by an order-independent digest per rank of the decoded rows."""
    from sahara_amd.dist import gather_compact_records, gather_hits, max_over_ranks, records_to_rows

    qoff = 2 * nreads * rank
    compact = hasattr(result, "recs")
    if compact:
        local = records_to_rows(result.recs, result.block_qid0 + np.uint64(qoff), result.block_end, rec_starts)
    else:
        h = result.to_hits()
        local = np.stack([h["qid"] + np.uint64(qoff), h["seq_id"], h["pos"], h["err"]], 1).astype(np.uint64)
    barrier()
    t = time.perf_counter()
    if compact:
        parts = gather_compact_records(result.recs, result.block_qid0, result.block_end, qoff, device=device)
    else:
        parts = gather_hits(local, 0, device=device)
    barrier()
    el = max_over_ranks(time.perf_counter() - t, device=device)
    mine = torch.tensor([rows_digest(local)], dtype=torch.int64, device=device)
    digs = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(digs, mine)
    ok, nrec = None, None
    if rank == 0:
        if compact:
            rows = [records_to_rows(r, q0, e, rec_starts) for r, q0, e in parts]
            nrec = sum(len(r) for r, _, _ in parts)
            ok = all(rows_digest(x) == int(d.item()) for x, d in zip(rows, digs))
            ok = ok and all(len(x) == 0 or int(x[:, 0].min()) >= 2 * nreads * r for r, x in enumerate(rows))
        else:
            nrec = len(parts)
            ok = rows_digest(parts) % (1 << 64) == sum(int(d.item()) % (1 << 64) for d in digs) % (1 << 64)
    rec_bytes = 8 if compact else 32
    out = {"ms": round(el * 1e3, 2), "verified": ok,
           "collective": ("all_gather of counts + gather of the 8-B compact records and of the block tables to rank "
                          "0 (RCCL over xGMI); host -> device before, device -> host on rank 0 after, inside the "
                          "timing") if compact else "all_gather of (qid, seq_id, pos, e) rows (RCCL over xGMI)",
           "source": "the last timed call's result (host memory)"}
    if rank == 0:
        out.update({"records": nrec, "bytes": nrec * rec_bytes, "GBs_into_rank0": round(nrec * rec_bytes / el / 1e9, 1)})
    return out


def rows_digest(rows):
    """hits_digest over (n, 4) u64 rows (qid, seq_id, pos, e), as a signed
    int64 (a torch tensor's word)."""
    rows = np.asarray(rows, np.uint64).reshape(-1, 4)
    h = np.zeros(len(rows), HIT_DTYPE_BENCH)
    h["qid"], h["seq_id"], h["pos"], h["err"] = rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3]
    d = hits_digest(h)
    return d - (1 << 64) if d >= (1 << 63) else d


def origin_recall(h, origin, k):
    """Fraction of reads with a forward-strand hit (qid 2i) in the record they
    were sampled from, within k positions of the sampled start (a leading
    I or D moves the reported start by up to k) and with at most k errors."""
    fwd = h[(h["qid"] & np.uint64(1)) == 0]
    read = (fwd["qid"] >> np.uint64(1)).astype(np.int64)
    ok = ((fwd["seq_id"].astype(np.uint64) == origin[read, 0]) & (fwd["err"] <= k) &
          (np.abs(fwd["pos"].astype(np.int64) - origin[read, 1].astype(np.int64)) <= k))
    found = np.zeros(len(origin), bool)
    found[read[ok]] = True
    return float(found.mean())


def verify_index(idx, flat, lens, torch, dev, W=21):
    """verify_index_part for every part of the index (one part unless the
    text exceeds 32-bit rows), each against its own records' text."""
    nparts = idx.info()["n_parts"]
    out, r0, off = None, 0, 0
    lens = np.asarray(lens, np.uint64)
    for p in range(nparts):
        idx.select_part(p)
        nr = idx.part_info(p)["n_records"]
        plen = lens[r0:r0 + nr]
        span = int(plen.sum())
        res = verify_index_part(idx, flat[off:off + span], plen, torch, dev, W)
        if out is None:
            out = res
        else:
            out["sa_probe_ok"] = out["sa_probe_ok"] and res["sa_probe_ok"]
            out["index_checks"] = {k: out["index_checks"][k] and v for k, v in res["index_checks"].items()}
            out["index_check_rows"] += res["index_check_rows"]
            out["index_check_s"] = round(out["index_check_s"] + res["index_check_s"], 1)
            out["index_check_max_lcp_blocks"] = max(out["index_check_max_lcp_blocks"], res["index_check_max_lcp_blocks"])
        r0 += nr
        off += span
    idx.select_part(0)
    out["index_parts"] = nparts
    return out


def verify_index_part(idx, flat, lens, torch, dev, W=21):
    """Checks the GPU-built forward index of the bench text row by row,
    independently of the code that built it (torch ops on the device):

    - the suffix array is strictly increasing in suffix order over all n rows
      (adjacent suffixes compared 21 symbols at a time as 63-bit keys; '$' is
      rank 0 and a suffix that ends sorts before its extensions, as
      oracle/oracle.cpp suffixArray) with every entry < n — so it is the
      suffix array of the text;
    - BWT[i] == T[SA[i] - 1] for every row (index.cpp:87's BWT);
    - the sampled-row bits and the samples are exactly the rows whose text
      position is a multiple of the rate within its record or a delimiter,
      in row order, i.e. the row -> position -> row
      round trip of LocateLinear;
    - C[] and the symbol counts of the reverse BWT match the text's."""
    t0 = time.time()
    inf = idx.part_info()
    n, rate = int(inf["n"]), int(inf["sampling_rate"])
    ex = idx.export()
    sa_h = idx.export_sa()
    lens64 = np.asarray(lens, np.int64)
    starts = np.concatenate([[0], np.cumsum(lens64 + 1)]).astype(np.int64)
    mask = 0xFFFFFFFF
    # text ranks + 1 ('$' = 1, past the end = 0)
    Tp = torch.zeros(n + 4 * W, dtype=torch.uint8, device=dev)
    off = 0
    for r, L in enumerate(lens64.tolist()):
        s = int(starts[r])
        Tp[s:s + L] = torch.from_numpy(flat[off:off + L]).to(dev) + 1
        Tp[s + L] = 1
        off += L
    CH = 1 << 27
    K = torch.empty(n + 2 * W, dtype=torch.int64, device=dev)
    for s in range(0, n + 2 * W, CH):
        e = min(n + 2 * W, s + CH)
        kk = torch.zeros(e - s, dtype=torch.int64, device=dev)
        for j in range(W):
            kk = (kk << 3) | Tp[s + j:e + j].to(torch.int64)
        K[s:e] = kk
    del kk
    sa_d = torch.from_numpy(sa_h.view(np.int32)).to(dev)
    del sa_h
    bwt_d = torch.from_numpy(ex["bwt_f"]).to(dev)
    words = torch.from_numpy(ex["sampled"].view(np.int64)).to(dev)
    samples_d = torch.from_numpy(ex["samples"].view(np.int32)).to(dev)
    starts_d = torch.from_numpy(starts).to(dev)
    ok = {"sa_sorted": True, "sa_in_range": True, "bwt": True, "samples": True}
    seen = 0
    max_lcp = 0
    for s in range(0, n, CH):
        e = min(n, s + CH)
        a = sa_d[s:e].to(torch.int64) & mask
        if bool((a >= n).any()):
            ok["sa_in_range"] = False
            break
        prev = torch.where(a == 0, torch.full_like(a, n - 1), a - 1)
        if not torch.equal(Tp[prev].to(torch.int16) - 1, bwt_d[s:e].to(torch.int16)):
            ok["bwt"] = False
        del prev
        # sampled rows: in-record offset a multiple of the rate, or the delimiter
        rec = torch.searchsorted(starts_d, a, right=True) - 1
        offr = a - starts_d[rec]
        want = ((offr % rate) == 0) | (offr == starts_d[rec + 1] - starts_d[rec] - 1)
        rows = torch.arange(s, e, device=dev, dtype=torch.int64)
        bit = ((words[rows >> 6] >> (rows & 63)) & 1).bool()
        if not torch.equal(bit, want):
            ok["samples"] = False
        pos = a[want]
        if not torch.equal(samples_d[seen:seen + pos.numel()].to(torch.int64) & mask, pos):
            ok["samples"] = False
        seen += pos.numel()
        del rec, offr, want, rows, bit, pos
        # adjacent rows (i, i + 1) for i in [s, min(e, n - 1))
        b = sa_d[s + 1:min(n, e + 1)].to(torch.int64) & mask
        x = a[:b.numel()]
        d = 0
        while x.numel():
            ka = K[torch.clamp(x + d, max=n)]
            kb = K[torch.clamp(b + d, max=n)]
            if bool((ka > kb).any()):
                ok["sa_sorted"] = False
                break
            eq = ka == kb
            x, b = x[eq], b[eq]
            d += W
            if d > 200 * W:
                ok["sa_sorted"] = False
                break
        max_lcp = max(max_lcp, d)
        del a, b, x
    ok["samples"] = ok["samples"] and seen == len(ex["samples"])
    cnt = torch.bincount(Tp[:n], minlength=8).cpu().numpy()[1:].astype(np.uint64)  # per rank
    sigma = int(inf["sigma"])
    C = np.concatenate([[0], np.cumsum(cnt[:sigma])]).astype(np.uint64)
    ok["C"] = bool(np.array_equal(C, ex["C"][:sigma + 1].astype(np.uint64)))
    rc = torch.bincount(torch.from_numpy(ex["bwt_r"]).to(dev), minlength=sigma).cpu().numpy()[:sigma].astype(np.uint64)
    ok["bwt_r_counts"] = bool(np.array_equal(rc, cnt[:sigma]))
    del Tp, K, sa_d, bwt_d, words, samples_d, starts_d
    torch.cuda.empty_cache()
    out = {"sa_probe_ok": all(ok.values()), "index_checks": ok, "index_check_rows": n,
           "index_check_s": round(time.time() - t0, 1), "index_check_max_lcp_blocks": max_lcp // W}
    return out


def hits_digest(h):
    """Host restatement of search.hip kDigest (order-independent sum of a
    64-bit mix per record) over a HIT_DTYPE array."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def mix64(x):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xbf58476d1ce4e5b9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94d049bb133111eb)
        return x ^ (x >> np.uint64(31))

    acc = 0
    with np.errstate(over="ignore"):
        for s in range(0, len(h), 1 << 24):
            b = h[s:s + (1 << 24)]
            inner = mix64((b["seq_id"].astype(np.uint64) << np.uint64(40)) ^ (b["pos"] << np.uint64(4)) ^
                          b["err"].astype(np.uint64))
            v = mix64((b["qid"] * np.uint64(0x9E3779B97F4A7C15)) ^ inner)
            acc = (acc + int(v.sum(dtype=np.uint64))) & int(M)
    return acc


def pcie_inclusive(search, idx, nreads, steps, warmup, world, barrier, local_hits, local_digest, path):
    """`search()` from host ranks to located hits in host memory (SURVEY §8(d)'s
    search wall time), timed over `steps` calls after `warmup` calls. Each
    call's hit buffer is released (sahara_gpu_free) before the next, except
    the last one's, whose content is checked (after the timing) against the
    device-resident pass's digest."""
    n = 0
    for _ in range(warmup):
        h = search()
        n = len(h)
        del h
    barrier()
    t0 = time.perf_counter()
    acc = {"stage_ms": 0.0, "total_ms": 0.0, "output_ms": 0.0}
    h = None
    for _ in range(steps):
        h = None
        h = search()
        st = idx.stats()
        for kk in acc:
            acc[kk] += st[kk]
        n = len(h)
    barrier()
    el = time.perf_counter() - t0
    same_digest = hits_digest(h.to_hits() if hasattr(h, "to_hits") else h) == local_digest
    del h
    if world > 1:
        from sahara_amd.dist import max_over_ranks
        el = max_over_ranks(el, device="cuda")
    return {"reads_per_s": round(nreads * world * steps / el, 1), "ms_per_step": round(el * 1e3 / steps, 2),
            "steps": steps, "warmup": warmup, "hits": int(n),
            "same_hits": int(n) == int(local_hits) and same_digest,
            "stage_ms": round(acc["stage_ms"] / steps, 2), "search_ms": round(acc["total_ms"] / steps, 2),
            "output_ms": round(acc["output_ms"] / steps, 2),
            "upload_chunks_2_4_8_bits": list(idx.stats()["upload_chunks"]), "path": path}


def reference_path(idx, ref_cnt, nreads, pat_bytes, steps, world, barrier, config):
    """The reference's execution model on the same staged reads: every DFS node
    ranked on the FM-index from the root (kSearchFM, no k-mer table, no text
    phase) and LocateLinear's LF walk to the rate-16 samples (kLocate<false>).
    Its roofline is SURVEY §8(d)'s B_read over HBM peak."""
    idx.set_mode(verify=False, locate_sa=False)
    try:
        idx.run()
        barrier()
        t0 = time.perf_counter()
        launches = 0
        for _ in range(steps):
            idx.run()
            launches += idx.stats()["search_launches"]
        barrier()
        el = time.perf_counter() - t0
    finally:
        idx.set_mode(verify=True, locate_sa=True)
    if world > 1:
        from sahara_amd.dist import max_over_ranks
        el = max_over_ranks(el, device="cuda")
    rps = nreads * world * steps / el
    fm_bytes = 64.0 * ref_cnt["ext_lines"] + pat_bytes        # per step: Occ lines + query bytes
    loc_bytes = 64.0 * (ref_cnt["lf_steps"] + ref_cnt["hits"])  # LF lines + one SA-sample line per row
    b_read = (fm_bytes + loc_bytes) / nreads
    per_gpu = b_read * rps / world / 1e9
    out = {"reads_per_s": round(rps, 1), "ms_per_step": round(el * 1e3 / steps, 2), "steps": steps,
           "B_read": round(b_read, 1),
           "roofline": {"bound": "hbm", "achieved": round(per_gpu, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(per_gpu / HBM_PEAK_GBS, 4),
                        "basis": "SURVEY 8(d) B_read (64 B per Occ line ranked, per LF step and per SA-sample "
                                 "line, + query bytes) x reads/s per GPU, over the whole step"},
           "kernels": {"kSearchFM": {"launches_per_step": launches // steps,
                                     "algorithmic_bytes_per_step": round(fm_bytes)},
                       "kLocate": {"algorithmic_bytes_per_step": round(loc_bytes)}},
           "mode": "set_mode(verify=0, locate_sa=0)"}
    # per-launch durations and FETCH_SIZE of both kernels from the committed
    # profile of this mode (tools/traffic_ref.sh: rocprofv3 kernel trace +
    # FETCH_SIZE pass of `bench.py --execution reference`)
    tj = os.path.join(ROOT, "profiles", f"traffic_{config}_ref.json")
    if os.path.exists(tj):
        tr = json.load(open(tj))
        for kn in ("kSearchFM", "kLocate"):
            if kn in tr:
                kk = out["kernels"][kn]
                per_step = kk["algorithmic_bytes_per_step"]
                kk.update({"avg_launch_us": tr[kn]["avg_launch_us"], "launches_per_step_profiled":
                           tr[kn]["dispatches"] / tr.get("steps", 1),
                           "traffic_bytes_per_launch": tr[kn]["bytes_per_launch"],
                           "traffic_GBs": tr[kn]["traffic_GBs"]})
                launches_k = tr[kn]["dispatches"] / tr.get("steps", 1)
                alg = per_step / max(launches_k, 1)
                kk["algorithmic_GBs"] = round(alg / (tr[kn]["avg_launch_us"] / 1e6) / 1e9, 1)
                kk["frac"] = round(kk["algorithmic_GBs"] / HBM_PEAK_GBS, 4)
        out["traffic_source"] = os.path.relpath(tj, ROOT)
    return out


def cpu_baseline(sa, idx, pats, scheme, edit, nreads, target_s, timed_hits=None):
    """Time the CPU restatement on a bounded sample; check GPU == CPU on it:
    `timed_hits` (the last timed call's hits, decoded; sorted by qid) cut to
    the sample's queries — the headline call at its default chunking and
    batching — and the patterns call (sahara_gpu_search) over the sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    t = time.time()
    # one oracle index per part of the GPU index (a multi-part index: the
    # sample is searched in every part, seq_ids offset by the part's first
    # record, as capi.cpp run merges them)
    refs, rec0 = [], 0
    for p in range(idx.info()["n_parts"]):
        idx.select_part(p)
        ex = idx.export()
        refs.append((O.Index.from_parts(ex["sigma"], ex["n"], ex["rec_lens"], ex["rate"], ex["bwt_f"], ex["bwt_r"],
                                        ex["sampled"], ex["samples"]), rec0))
        rec0 += len(ex["rec_lens"])
        del ex
    idx.select_part(0)
    log(f"cpu baseline: oracle index loaded, {len(refs)} part(s) ({time.time()-t:.1f}s)")
    threads = host_threads()

    def cpu_search(q, nthreads):
        out = []
        for ref, r0 in refs:
            h, _ = ref.search(q, scheme, edit=edit, nthreads=nthreads)
            h = np.asarray(h, np.uint64).reshape(-1, 4)
            h[:, 1] += np.uint64(r0)
            out.append(h)
        return np.concatenate(out)

    # calibrate: grow the sample until it runs >= 1 s, then scale to ~target_s
    n = min(1000, nreads)
    while True:
        t = time.perf_counter()
        cpu_search(pats[: 2 * n], threads)
        dt = time.perf_counter() - t
        if dt >= 1.0 or n >= nreads:
            break
        n = min(nreads, n * 4)
    n2 = int(min(nreads, max(n, n * target_s / max(dt, 1e-3))))
    t = time.perf_counter()
    hits = cpu_search(pats[: 2 * n2], threads)
    dt = time.perf_counter() - t
    rate = n2 / dt
    # single-thread figure (the reference's execution model, search.cpp:221-241)
    n1 = max(20, min(n2, int(n2 / threads / 4)))
    t = time.perf_counter()
    cpu_search(pats[: 2 * n1], 1)
    rate1 = n1 / (time.perf_counter() - t)
    # parity on the sample
    h = hits
    want = h[np.lexsort((h[:, 3], h[:, 2], h[:, 1], h[:, 0]))]

    def rows_of(g):
        return np.stack([g["qid"], g["seq_id"], g["pos"], g["err"]], 1).astype(np.uint64)

    gpu_hits = sa.search(idx, pats[: 2 * n2], scheme, edit=edit)
    from_gpu = rows_of(gpu_hits)
    parity_patterns = bool(len(want) == len(from_gpu) and np.array_equal(want, from_gpu))
    parity = None
    if timed_hits is not None:
        cut = int(np.searchsorted(timed_hits["qid"], np.uint64(2 * n2)))
        from_timed = rows_of(timed_hits[:cut])
        parity = bool(len(want) == len(from_timed) and np.array_equal(want, from_timed))
    log(f"cpu baseline: {n2} reads in {dt:.1f}s on {threads} threads = {rate:.0f} reads/s "
        f"(1 thread: {rate1:.0f} reads/s); GPU==CPU on sample: timed call {parity}, patterns call {parity_patterns}")
    return {"value": round(rate, 1), "unit": "reads/s", "cores": threads, "kind": "port",
            "sample": f"first {n2} reads (+RC) of the same workload, {dt:.1f}s; "
                      f"1-thread rate {rate1:.1f} reads/s on {n1} reads; host CPU: {cpu_model()}",
            "single_thread_value": round(rate1, 1),
            "parity_on_sample": parity if parity is not None else parity_patterns,
            "parity_source": ("the last timed call's records (sahara_gpu_search_packed_compact at its default chunks "
                              "and batches), cut to the sample's queries") if parity is not None
                             else "sahara_gpu_search over the sample",
            "parity_patterns_call": parity_patterns, "index_parts": len(refs)}


if __name__ == "__main__":
    main()
