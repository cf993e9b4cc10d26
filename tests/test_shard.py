"""`sahara search --gpus N` query sharding (sahara_amd/cli/shard.h), run on CPU.

The product's own shard function is compiled into a small shared library and
called through ctypes. Each shard's queries are rebuilt the way the device
path builds them (reads [r0, r1), reverse complements interleaved, cut at
q1 - q0, qids shifted by q0), searched with the CPU restatement, and
gathered; the result must equal one search over the whole interleaved,
--limit_queries-cut list (search.cpp:111-127). The two-rank variant runs the
same shards as gloo ranks and gathers with sahara_amd.dist.gather_hits.
"""
import ctypes
import os
import socket
import subprocess
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import hits_as_rows, mutate_reads, random_records

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#include "shard.h"
extern "C" void query_shard(size_t nq, size_t per, unsigned devices, unsigned g, size_t* out) {
    const sahara_cli::QueryShard s = sahara_cli::queryShard(nq, per, devices, g);
    out[0] = s.r0; out[1] = s.r1; out[2] = s.q0; out[3] = s.q1;
}
'''


@pytest.fixture(scope="module")
def shard_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("shard")
    (d / "s.cpp").write_text(SRC)
    so = d / "libshard.so"
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "sahara_amd", "cli"),
                    str(d / "s.cpp"), "-o", str(so)], check=True)
    return str(so)


def shard(lib_path, nq, per, devices, g):
    L = ctypes.CDLL(lib_path)
    out = (ctypes.c_size_t * 4)()
    L.query_shard(ctypes.c_size_t(nq), ctypes.c_size_t(per), ctypes.c_uint(devices), ctypes.c_uint(g), out)
    return tuple(out)


def _rc(reads):
    comp = np.array([0, 5, 3, 2, 4, 1], np.uint8)
    return comp[reads[:, ::-1]]


def shard_patterns(reads, per, r0, r1, q0, q1):
    """What sahara_gpu_search_reads stages for one shard."""
    sub = reads[r0:r1]
    if per == 1:
        pats = sub
    else:
        pats = np.empty((2 * len(sub), reads.shape[1]), np.uint8)
        pats[0::2] = sub
        pats[1::2] = _rc(sub)
    return pats[: q1 - q0]


def full_list(reads, per, nq):
    return shard_patterns(reads, per, 0, len(reads), 0, nq)


def test_shards_partition_the_query_list(shard_lib):
    for nq in (1, 2, 3, 7, 100, 101, 2 * 12345 - 1):
        for per in (1, 2):
            for dev in (1, 2, 3, 8):
                prev_r = prev_q = 0
                for g in range(dev):
                    r0, r1, q0, q1 = shard(shard_lib, nq, per, dev, g)
                    assert (r0, q0) == (prev_r, prev_q) and r1 >= r0 and q1 >= q0
                    assert q1 - q0 <= per * (r1 - r0)
                    prev_r, prev_q = r1, q1
                assert prev_q == nq and prev_r == (nq + per - 1) // per


@pytest.mark.parametrize("per,limit", [(2, None), (2, 77), (1, None), (1, 40)])
def test_sharded_search_equals_single_search(shard_lib, per, limit):
    import oracle as O
    rng = np.random.default_rng(5)
    recs = random_records(rng, [4000, 2500], 6, repeats=True)
    reads = mutate_reads(rng, recs, 60, 36, 2)
    nq = per * len(reads) if limit is None else min(limit, per * len(reads))
    idx = O.Index.build(recs, 6, 16)
    sch = O.scheme("h2-k2", 0, 2, 36)
    want = hits_as_rows(idx.search(full_list(reads, per, nq), sch)[0])
    for dev in (2, 3, 8):
        got = []
        for g in range(dev):
            r0, r1, q0, q1 = shard(shard_lib, nq, per, dev, g)
            if r0 == r1:
                continue
            h = np.asarray(idx.search(shard_patterns(reads, per, r0, r1, q0, q1), sch)[0], np.uint64).reshape(-1, 4)
            h[:, 0] += np.uint64(q0)
            got.append(h)
        assert np.array_equal(hits_as_rows(np.concatenate(got)), want), dev


def _rank(rank, world, port, lib_path, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import oracle as O
    from sahara_amd.dist import gather_hits

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(5)
        recs = random_records(rng, [4000, 2500], 6, repeats=True)
        reads = mutate_reads(rng, recs, 60, 36, 2)
        nq = 2 * len(reads) - 3  # --limit_queries cuts inside the last rank's shard
        r0, r1, q0, q1 = shard(lib_path, nq, 2, world, rank)
        idx = O.Index.build(recs, 6, 16)
        h, _ = idx.search(shard_patterns(reads, 2, r0, r1, q0, q1), O.scheme("h2-k2", 0, 2, 36))
        allh = gather_hits(h, qid_offset=q0)
        if rank == 0:
            np.save(os.path.join(outdir, "g.npy"), allh)
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_over_gloo(shard_lib):
    import oracle as O
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(2, port, shard_lib, d), nprocs=2, join=True, start_method="spawn")
        got = np.load(os.path.join(d, "g.npy"))
    rng = np.random.default_rng(5)
    recs = random_records(rng, [4000, 2500], 6, repeats=True)
    reads = mutate_reads(rng, recs, 60, 36, 2)
    nq = 2 * len(reads) - 3
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(full_list(reads, 2, nq), O.scheme("h2-k2", 0, 2, 36))[0])
    assert len(want) and np.array_equal(hits_as_rows(got), want)
