"""C4's multi-device path (BASELINE configs[3]) executed on the one
GPU a test box has: SAHARA_DEVICE_MAP maps every context of `sahara search
--gpus N` (and of the ctypes binding) to device 0, so the threaded index
load, the read shards (cli/shard.h), the concurrent searches of several
contexts (each with its own streams, pinned rings and packing pool, sharing
the process-wide pinned hit pool) and the concatenation in qid order all
run. The output must equal the single-process reference order and multiset
(search.cpp:218-261): the golden hit files. No scaling is claimed here."""
import os
import threading

import numpy as np
import pytest

import sahara_amd as sa
from helpers import hits_as_rows
from test_cli import read_hits, run
from test_golden import CASES, GOLD, IDX, expected, limit_rows, patterns, read_fasta, SIGMA


def _env(n):
    return {"SAHARA_DEVICE_MAP": ",".join(["0"] * n)}


def run_env(env, *args):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return run(*args)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def device_lines(so):
    return [ln for ln in so.splitlines() if ln.startswith("  device ")]


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2, 3, 8])
@pytest.mark.parametrize("name", ["a_lev_k2", "a_ham_k2", "a_best_k2", "a_lev_k2_pigeon_norev", "b_lev_k3"])
def test_cli_gpus_n_equals_golden(gpus, name, tmp_path, gpu_device):
    c = CASES[name]
    args = ["-e", c["k"], "-g", c["generator"], "-d", c["metric"], "-m", c["mode"], "--emit-errors"]
    if not c["reverse"]:
        args.append("--no-reverse")
    q = os.path.join(GOLD, f"reads_{c['fixture']}.fa")
    i = os.path.join(GOLD, IDX[c["fixture"]])
    one, many = tmp_path / "one.txt", tmp_path / "many.txt"
    rc, so1, err = run("search", "-q", q, "-i", i, "-o", one, *args)
    assert rc == 0, err
    rc, so, err = run_env(_env(gpus), "search", "-q", q, "-i", i, "-o", many, "--gpus", gpus, *args)
    assert rc == 0, err
    got = read_hits(many, 4)
    # same lines in the same order as one device (shards concatenate in qid order)
    assert np.array_equal(got, read_hits(one, 4))
    assert np.array_equal(hits_as_rows(got), expected(name))
    assert f"  number of hits:      {c['hits']:>10}" in so
    lines = device_lines(so)
    assert [ln.split(":")[0].strip() for ln in lines] == [f"device {g}" for g in range(gpus)]
    per_dev = [int(ln.rsplit("hits ", 1)[1]) for ln in lines]
    assert sum(per_dev) == c["hits"]
    # each device's hits are exactly its shard's queries
    per = 2 if c["reverse"] else 1
    nreads = c["patterns"] // per
    for g in range(gpus):
        r0, r1 = nreads * g // gpus, nreads * (g + 1) // gpus
        sel = (got[:, 0] >= per * r0) & (got[:, 0] < per * r1)
        assert int(sel.sum()) == per_dev[g]
    assert device_lines(so1) == []


@pytest.mark.gpu
@pytest.mark.parametrize("limit", [111, 40, 3])
def test_cli_gpus_limit_queries_cuts_last_shard(limit, tmp_path, gpu_device):
    """--limit_queries 111 leaves 56 reads (the last one forward only): the cut
    falls inside device 2's shard; 3 leaves two reads, none for device 0;
    --max_hits on top."""
    out = tmp_path / "h.txt"
    rc, so, err = run_env(_env(3), "search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i",
                          os.path.join(GOLD, IDX["a"]), "-e", 2, "--limit_queries", limit, "--max_hits", 3,
                          "--emit-errors", "-o", out, "--gpus", 3)
    assert rc == 0, err
    want = expected("a_lev_k2")
    want = limit_rows(want[want[:, 0] < limit], 3)
    assert np.array_equal(hits_as_rows(read_hits(out, 4)), want)
    fwd = limit // 2  # search.cpp:150-151: queries.size() / 2, the odd one counted backward
    assert f"fwd queries: {fwd}\nbwd queries: {limit - fwd}\n" in so
    assert len(device_lines(so)) == 3


@pytest.mark.gpu
def test_cli_device_map_without_entry_is_loud(tmp_path, gpu_device):
    rc, _, err = run_env(_env(1), "search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                         "-e", 1, "-o", tmp_path / "h.txt", "--gpus", 2)
    assert rc == 1 and "SAHARA_DEVICE_MAP has no entry for device 1" in err


def _proc_status():
    got = {}
    for line in open("/proc/self/status"):
        k, _, v = line.partition(":")
        if k in ("Threads", "VmLck", "VmPin", "VmRSS"):
            got[k] = v.strip()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8])
def test_concurrent_contexts_on_shards(gpu_device, monkeypatch, n):
    """n contexts searched from n host threads at once (ctypes drops the GIL
    in the calls), each on its own shard of the reads, several rounds (the
    second and later draw their hit sinks from the shared pinned pool), half
    of them through the packed-reads compact call: the concatenation equals
    the golden multiset, every round. At n = 8 (C4's host side: eight packing
    pools, eight pinned rings, one shared hit pool under contention) the
    process's thread count and locked memory are printed."""
    monkeypatch.setenv("SAHARA_DEVICE_MAP", ",".join(["0"] * n))
    monkeypatch.setenv("SAHARA_PIN_MIN", "0")  # every hit buffer pinned and pooled
    monkeypatch.setenv("SAHARA_BATCH", "17")   # several batches per call: the pipeline's threads
    c = CASES["a_lev_k2"]
    reads = np.array(read_fasta(os.path.join(GOLD, "reads_a.fa"), SIGMA["a"]))
    m = reads.shape[1]
    scheme = sa.search_scheme("h2-k2", 0, c["k"], m)
    before = _proc_status()
    ctx = [sa.BiFMIndex.load(os.path.join(GOLD, IDX["a"]), device=g) for g in range(n)]
    for g in ctx:
        pl = g.placement()
        assert pl["device"] == 0
        assert pl["numa_node"] >= -1 and pl["n_cpus"] >= 0
        assert pl["n_cpus"] == 0 or pl["numa_node"] >= 0
    bounds = [len(reads) * g // n + (3 if 0 < g < n else 0) for g in range(n)] + [len(reads)]
    shards = [(bounds[g], bounds[g + 1]) for g in range(n)]
    packed = sa.pack_reads(reads, SIGMA["a"])
    want = expected("a_lev_k2")
    peak = {}
    for rnd in range(4):
        out, errs = [None] * n, []

        def work(g):
            try:
                r0, r1 = shards[g]
                if (g + rnd) % 2:
                    h = sa.search_packed_compact(ctx[g], packed.shard(r0, r1), scheme, edit=True)
                    rows = hits_as_rows(h.to_hits()).copy()
                    h.close()
                else:
                    rows = hits_as_rows(sa.search_reads(ctx[g], reads[r0:r1], scheme, edit=True)).copy()
                rows[:, 0] += 2 * r0
                out[g] = rows
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=work, args=(g,)) for g in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        assert np.array_equal(np.concatenate(out), want)
        peak = _proc_status()
    print(f"\n[{n} contexts] before: {before} after the searches: {peak}")
    for g in ctx:
        g.close()


@pytest.mark.gpu
def test_cli_gpus_8_medium_equals_one(tmp_path, gpu_device):
    """`sahara search --gpus 8` on a medium case (2 Mbp in 24 records, 20k
    reads of 101 bp with 2 errors, so device shards start inside a byte of
    the packed reads) writes the file `--gpus 1` writes, and both equal the
    oracle's multiset."""
    import oracle as O
    from test_packed import _write_fasta
    lens = np.full(24, 2_000_000 // 24, np.uint64)
    flat, lens = sa.synth_reference(lens, sigma=6, seed=5)
    reads = sa.synth_reads(flat, lens, 20_000, 101, 2, sigma=6, seed=6)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    recs = [flat[offs[i]:offs[i + 1]] for i in range(len(lens))]
    ref = tmp_path / "ref.fa"
    _write_fasta(ref, recs, width=80)
    q = tmp_path / "reads.fa"
    _write_fasta(q, reads, width=80)
    rc, _, err = run("index", ref)
    assert rc == 0, err
    one, many = tmp_path / "one.txt", tmp_path / "many.txt"
    rc, so1, err = run("search", "-q", q, "-i", f"{ref}.idx", "-e", 2, "--emit-errors", "-o", one)
    assert rc == 0, err
    rc, so, err = run_env(_env(8), "search", "-q", q, "-i", f"{ref}.idx", "-e", 2, "--emit-errors", "-o", many,
                          "--gpus", 8)
    assert rc == 0, err
    assert open(one).read() == open(many).read()
    assert len(device_lines(so)) == 8
    pats = sa.interleave_rc(reads, 6)
    want, _ = O.Index.build(recs, 6, 16).search(pats, sa.search_scheme("h2-k2", 0, 2, 101), edit=True, nthreads=8)
    assert np.array_equal(hits_as_rows(read_hits(many, 4)), hits_as_rows(want))


@pytest.mark.gpu
def test_numa_binding_can_be_turned_off(gpu_device, monkeypatch):
    monkeypatch.setenv("SAHARA_NUMA", "0")
    g = sa.BiFMIndex.load(os.path.join(GOLD, IDX["a"]))
    assert g.placement() == {"device": 0, "numa_node": -1, "n_cpus": 0}
    g.close()
