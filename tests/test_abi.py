"""The C-ABI library loads and exports every symbol include/sahara_hip.h
declares; host-side utilities behave (no GPU compute here)."""
import ctypes
import os
import re

import numpy as np

import sahara_amd as sa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "sahara_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sahara_[a-z_0-9]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    assert len(names) >= 20
    L = ctypes.CDLL(sa.library_path())
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python mirror binds every one of them
    assert set(names) <= set(sa.EXPORTED), set(names) - set(sa.EXPORTED)


def test_library_is_gfx950_code_object():
    data = open(sa.library_path(), "rb").read()
    assert b"gfx950" in data


def test_synth_reference_deterministic():
    a, la = sa.synth_reference([1000, 37], sigma=6, seed=42)
    b, _ = sa.synth_reference([1000, 37], sigma=6, seed=42)
    c, _ = sa.synth_reference([1000, 37], sigma=6, seed=43)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert set(np.unique(a).tolist()) == {1, 2, 3, 5}
    d, _ = sa.synth_reference([64], sigma=5, seed=1)
    assert set(np.unique(d).tolist()) <= {1, 2, 3, 4}


def edit_distance(a, b):
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (a[i - 1] != b[j - 1]))
        prev = cur
    return prev[-1]


def test_synth_reads_follow_transcript_semantics():
    flat, lens = sa.synth_reference([3000, 2000], sigma=6, seed=42)
    reads, origin = sa.synth_reads(flat, lens, 200, 40, 2, sigma=6, seed=7, with_origin=True)
    again = sa.synth_reads(flat, lens, 200, 40, 2, sigma=6, seed=7)
    assert np.array_equal(reads, again)
    starts = [0] + np.cumsum(lens.astype(np.int64))[:-1].tolist()
    for i in range(0, 200, 7):
        rec, pos = int(origin[i, 0]), int(origin[i, 1])
        ref = flat[starts[rec] + pos: starts[rec] + pos + 44]
        # the read aligns to a prefix of the reference span with <= 2 edits
        best = min(edit_distance(reads[i].tolist(), ref[:L].tolist()) for L in range(38, 43))
        assert best <= 2


def test_synth_reads_substitutions_only():
    # Hamming workloads (C2): exactly k substitutions, no indels
    flat, lens = sa.synth_reference([3000, 2000], sigma=6, seed=42)
    reads, origin = sa.synth_reads(flat, lens, 300, 40, 0, sigma=6, seed=9, with_origin=True, substitutions=2)
    starts = [0] + np.cumsum(lens.astype(np.int64))[:-1].tolist()
    for i in range(300):
        rec, pos = int(origin[i, 0]), int(origin[i, 1])
        ref = flat[starts[rec] + pos: starts[rec] + pos + 40]
        assert int(np.count_nonzero(ref != reads[i])) == 2


def test_interleave_rc():
    r = np.array([[1, 2, 3, 5, 4], [5, 5, 1, 2, 2]], np.uint8)
    out = sa.interleave_rc(r, sigma=6)
    assert out.tolist() == [[1, 2, 3, 5, 4], [4, 1, 2, 3, 5], [5, 5, 1, 2, 2], [3, 3, 5, 1, 1]]
    r4 = np.array([[1, 2, 3, 4]], np.uint8)
    assert sa.interleave_rc(r4, sigma=5).tolist() == [[1, 2, 3, 4], [1, 2, 3, 4]]


def test_generators_listed():
    g = sa.scheme_generators()
    assert "h2-k2" in g and "backtracking" in g and "pigeon" in g


def test_hit_arrays_are_zero_copy_views_freed_by_the_library():
    import ctypes as C
    import gc
    libc = C.CDLL(None)
    libc.malloc.restype = C.c_void_p
    libc.malloc.argtypes = [C.c_size_t]
    n = 5
    ptr = libc.malloc(n * sa.HIT_DTYPE.itemsize)
    src = np.zeros(n, sa.HIT_DTYPE)
    src["qid"] = np.arange(n) * 3
    src["pos"] = 7
    C.memmove(ptr, src.ctypes.data, src.nbytes)
    a = sa._hits_array(C.c_void_p(ptr), n)
    assert a.dtype == sa.HIT_DTYPE and a.ctypes.data == ptr
    assert a["qid"].tolist() == [0, 3, 6, 9, 12] and (a["pos"] == 7).all()
    b = a[1:3]  # views keep the buffer alive
    del a
    gc.collect()
    assert b["qid"].tolist() == [3, 6]
    del b
    gc.collect()
    assert len(sa._hits_array(C.c_void_p(None), 0)) == 0
