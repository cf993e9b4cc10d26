"""ctypes wrapper around oracle/liboracle.so — the CPU restatement.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py. The product (sahara_amd/) never imports it.
See oracle/oracle.h for what each entry point restates (reference file:line).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("nodes", "rank_nodes", "ext_lines", "leaves", "rows", "lf_steps")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def lib():
    global _LIB
    if _LIB is None:
        # ORACLE_LIB: another build of the same restatement (the sanitizer build, tools/asan_cpu_tests.sh)
        path = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} missing (run `make -C oracle`)")
        L = C.CDLL(path)
        L.orc_build.restype = C.c_void_p
        L.orc_build.argtypes = [u8p, u64p, C.c_uint64, C.c_uint32, C.c_uint32]
        L.orc_from_parts.restype = C.c_void_p
        L.orc_from_parts.argtypes = [C.c_uint32, C.c_uint64, u64p, C.c_uint64, C.c_uint32,
                                     u8p, u8p, u64p, u32p, C.c_uint64]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_size.restype = C.c_uint64
        L.orc_size.argtypes = [C.c_void_p]
        L.orc_nsamples.restype = C.c_uint64
        L.orc_nsamples.argtypes = [C.c_void_p]
        L.orc_export.argtypes = [C.c_void_p, u8p, u8p, u32p, u64p, u32p, u64p]
        L.orc_write_idx.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_read_idx.restype = C.c_void_p
        L.orc_read_idx.argtypes = [C.c_char_p]
        L.orc_scheme.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_int,
                                 u32p, u32p, u32p, C.c_int]
        L.orc_scheme_complete.argtypes = [C.c_char_p, C.c_int, C.c_int]
        L.orc_search.restype = C.c_int64
        L.orc_search.argtypes = [C.c_void_p, u8p, C.c_uint64, C.c_uint32, u32p, u32p, u32p,
                                 C.c_uint32, C.c_int, C.c_int, C.POINTER(u64p), C.POINTER(Counters)]
        L.orc_search_cursors.restype = C.c_int64
        L.orc_search_cursors.argtypes = [C.c_void_p, u8p, C.c_uint64, C.c_uint32, u32p, u32p, u32p,
                                         C.c_uint32, C.c_int, C.POINTER(u64p)]
        L.orc_bruteforce.restype = C.c_int64
        L.orc_bruteforce.argtypes = [u8p, u64p, C.c_uint64, u8p, C.c_uint64, C.c_uint32,
                                     C.c_uint32, C.c_int, C.POINTER(u64p)]
        L.orc_free_buf.argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def _take(ptr, n, width=4):
    arr = np.ctypeslib.as_array(ptr, shape=(max(n, 1) * width,))[: n * width].copy()
    lib().orc_free_buf(ptr)
    return arr.reshape(n, width)


class Index:
    """Bidirectional FM-index restated on the CPU (index.cpp:41-112)."""

    def __init__(self, handle, sigma, rec_lens):
        self.h = handle
        self.sigma = sigma
        self.rec_lens = np.asarray(rec_lens, dtype=np.uint64)

    @classmethod
    def build(cls, records, sigma=6, rate=16):
        recs = [np.asarray(r, dtype=np.uint8) for r in records]
        ranks = np.ascontiguousarray(np.concatenate(recs) if recs else np.zeros(0, np.uint8))
        lens = np.array([len(r) for r in recs], dtype=np.uint64)
        h = lib().orc_build(_p(ranks, u8p), _p(lens, u64p), len(lens), sigma, rate)
        if not h:
            raise ValueError("orc_build failed")
        return cls(h, sigma, lens)

    @classmethod
    def from_parts(cls, sigma, n, rec_lens, rate, bwt_f, bwt_r, sampled_bits, samples):
        rec_lens = np.ascontiguousarray(rec_lens, dtype=np.uint64)
        bwt_f = np.ascontiguousarray(bwt_f, dtype=np.uint8)
        bwt_r = np.ascontiguousarray(bwt_r, dtype=np.uint8)
        sampled_bits = np.ascontiguousarray(sampled_bits, dtype=np.uint64)
        samples = np.ascontiguousarray(samples, dtype=np.uint32)
        h = lib().orc_from_parts(sigma, n, _p(rec_lens, u64p), len(rec_lens), rate,
                                 _p(bwt_f, u8p), _p(bwt_r, u8p), _p(sampled_bits, u64p),
                                 _p(samples, u32p), len(samples))
        return cls(h, sigma, rec_lens)

    @classmethod
    def read(cls, path):
        h = lib().orc_read_idx(str(path).encode())
        if not h:
            raise ValueError(f"cannot read index {path}")
        inst = cls(h, 0, [])
        return inst

    def write(self, path):
        if lib().orc_write_idx(self.h, str(path).encode()) != 0:
            raise IOError(path)

    @property
    def n(self):
        return int(lib().orc_size(self.h))

    def export(self, with_sa=True):
        n = self.n
        bf = np.zeros(n, np.uint8)
        br = np.zeros(n, np.uint8)
        sa = np.zeros(n, np.uint32) if with_sa else None
        sb = np.zeros(n // 64 + 1, np.uint64)
        ns = int(lib().orc_nsamples(self.h))
        smp = np.zeros(max(ns, 1), np.uint32)
        Cc = np.zeros(8, np.uint64)
        rc = lib().orc_export(self.h, _p(bf, u8p), _p(br, u8p), _p(sa, u32p) if with_sa else None,
                              _p(sb, u64p), _p(smp, u32p), _p(Cc, u64p))
        if rc != 0:
            raise ValueError("export failed")
        return dict(bwt_f=bf, bwt_r=br, sa=sa, sampled=sb, samples=smp[:ns], C=Cc)

    def search(self, pats, scheme, edit=True, nthreads=1, locate=True):
        """pats: (npat, m) uint8 ranks; scheme: (pi, l, u) arrays of shape (S, m).
        Returns (hits[n,4] = qid, seq_id, seq_pos, e; counters dict)."""
        pats = np.ascontiguousarray(pats, dtype=np.uint8)
        npat, m = pats.shape
        pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
        out = u64p()
        if locate:
            cnt = Counters()
            n = lib().orc_search(self.h, _p(pats, u8p), npat, m, _p(pi, u32p), _p(l, u32p),
                                 _p(u, u32p), pi.shape[0], int(edit), nthreads, C.byref(out),
                                 C.byref(cnt))
            return _take(out, n), cnt.as_dict()
        n = lib().orc_search_cursors(self.h, _p(pats, u8p), npat, m, _p(pi, u32p), _p(l, u32p),
                                     _p(u, u32p), pi.shape[0], int(edit), C.byref(out))
        return _take(out, n), None

    def __del__(self):
        try:
            if self.h:
                lib().orc_free(self.h)
        except Exception:
            pass


def scheme(generator, min_k, max_k, length, hamming=False):
    """Expanded search scheme (search.cpp:186-212, :226) -> (pi, l, u) of shape (S, length)."""
    L = lib()
    n = L.orc_scheme(generator.encode(), min_k, max_k, length, int(hamming), None, None, None, 0)
    if n < 0:
        raise ValueError(f"unknown generator {generator!r} or bad k")
    pi = np.zeros((n, length), np.uint32)
    l = np.zeros((n, length), np.uint32)
    u = np.zeros((n, length), np.uint32)
    rc = L.orc_scheme(generator.encode(), min_k, max_k, length, int(hamming),
                      _p(pi, u32p), _p(l, u32p), _p(u, u32p), n)
    if rc != n:
        raise ValueError(f"scheme expansion failed ({rc})")
    return pi, l, u


def scheme_complete(generator, min_k, max_k):
    return lib().orc_scheme_complete(generator.encode(), min_k, max_k) == 1


def bruteforce(records, pats, k, edit=True):
    recs = [np.asarray(r, dtype=np.uint8) for r in records]
    ranks = np.ascontiguousarray(np.concatenate(recs))
    lens = np.array([len(r) for r in recs], dtype=np.uint64)
    pats = np.ascontiguousarray(pats, dtype=np.uint8)
    out = u64p()
    n = lib().orc_bruteforce(_p(ranks, u8p), _p(lens, u64p), len(lens), _p(pats, u8p),
                             pats.shape[0], pats.shape[1], k, int(edit), C.byref(out))
    return _take(out, n)


def search_best(index, pats, schemes, nthreads=1):
    """search_ng21::search_best over per-exact-j schemes j = 0..k (search.cpp:233-241).

    Restated as: for every pattern, the located hits of the smallest j whose
    exact-j scheme (expand(generator(j, j), len), edit operations) reports any.
    schemes: list of (pi, l, u), index j = error count. Returns hits[n, 4]."""
    pats = np.ascontiguousarray(pats, dtype=np.uint8)
    todo = np.arange(pats.shape[0], dtype=np.uint64)
    out = []
    for sch in schemes:
        if len(todo) == 0:
            break
        h, _ = index.search(pats[todo], sch, edit=True, nthreads=nthreads)
        if len(h):
            h = h.copy()
            h[:, 0] = todo[h[:, 0]]
            out.append(h)
            todo = np.setdiff1d(todo, np.unique(h[:, 0]))
    if not out:
        return np.zeros((0, 4), np.uint64)
    return np.concatenate(out)
