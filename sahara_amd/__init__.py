"""sahara_amd — MI355X-native drop-in for sahara's search hot path.

Python mirror of the reference's operator interface for that path
(/root/reference/src/sahara/search.cpp:104-274), over the C ABI of
``sahara_amd/lib/libsahara_hip.so`` (include/sahara_hip.h):

    idx    = BiFMIndex.build(records, sigma=6)       # index.cpp:87  (GPU construction)
    idx    = BiFMIndex.load("ref.fa.idx")             # search.cpp:162-169
    scheme = search_scheme("h2-k2", 0, k, len)        # search.cpp:174-212 (+ :226 for ham)
    hits   = search(idx, queries, scheme, edit=True)  # search.cpp:218-250

There is no CPU fallback: every entry point runs the HIP kernels and fails
loudly when the extension or the GPU is missing.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

__all__ = [
    "BiFMIndex", "HIT_DTYPE", "search", "search_reads", "search_reads_compact", "CompactHits", "PackedReads",
    "pack_reads", "search_packed", "search_packed_compact", "read_fasta", "search_scheme", "scheme_parts",
    "scheme_generators",
    "scheme_counts", "synth_reference", "synth_reads", "interleave_rc", "load_fasta",
    "library_path", "lib", "SaharaError", "DNA5", "DNA4",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# ivsigma delimited alphabets: rank 0 is the delimiter '$'.
DNA5 = {"sigma": 6, "chars": "$ACGNT"}
DNA4 = {"sigma": 5, "chars": "$ACGT"}

HIT_DTYPE = np.dtype([("qid", "<u8"), ("seq_id", "<u4"), ("err", "<u4"), ("pos", "<u8")])

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class SaharaError(RuntimeError):
    pass


class HitBlocks(C.Structure):
    _fields_ = [("recs", C.POINTER(C.c_uint64)), ("n_hits", C.c_uint64), ("block_qid0", C.POINTER(C.c_uint64)),
                ("block_end", C.POINTER(C.c_uint64)), ("n_blocks", C.c_uint64),
                ("rec_starts", C.POINTER(C.c_uint64)), ("n_records", C.c_uint64)]


class FastaOut(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("n_symbols", C.c_uint64), ("offs", C.POINTER(C.c_uint64)),
                ("n_records", C.c_uint64), ("n_pos", C.POINTER(C.c_uint64)), ("n_count", C.c_uint64),
                ("bad", C.c_int), ("bad_char", C.c_uint32), ("bad_record", C.c_uint64), ("bad_pos", C.c_uint64),
                ("bad_id", C.c_char_p)]


class IndexInfo(C.Structure):
    _fields_ = [("sigma", C.c_uint32), ("sampling_rate", C.c_uint32), ("n", C.c_uint64),
                ("n_records", C.c_uint64), ("n_samples", C.c_uint64), ("device_bytes", C.c_uint64),
                ("n_parts", C.c_uint32), ("kmer_depth", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("patterns", C.c_uint64), ("batches", C.c_uint64), ("cursors", C.c_uint64),
                ("hits", C.c_uint64), ("search_ms", C.c_double), ("locate_ms", C.c_double),
                ("sort_ms", C.c_double), ("total_ms", C.c_double), ("nodes", C.c_uint64),
                ("rank_nodes", C.c_uint64), ("ext_lines", C.c_uint64), ("lf_steps", C.c_uint64),
                ("search_launches", C.c_uint32), ("search_grid", C.c_uint32),
                ("text_nodes", C.c_uint64), ("conversions", C.c_uint64), ("text_ms", C.c_double),
                ("fm_iterations", C.c_uint64), ("text_iterations", C.c_uint64), ("text_active", C.c_uint64),
                ("text_refills", C.c_uint64), ("text_cycles_refill", C.c_uint64),
                ("text_cycles_step", C.c_uint64), ("text_cycles_emit", C.c_uint64),
                ("text_compare_steps", C.c_uint64), ("text_grid", C.c_uint32), ("pipelined", C.c_uint32),
                ("seed_ms", C.c_double), ("text_steps", C.c_uint64), ("stage_ms", C.c_double),
                ("output_ms", C.c_double), ("text_launches", C.c_uint64),
                ("upload_chunks", C.c_uint64 * 3), ("text_pos_tasks", C.c_uint64),
                ("text_stolen", C.c_uint64), ("reserved", C.c_uint64 * 8)]

    def as_dict(self):
        return {n: (list(v) if isinstance(v, C.Array) else v) for n, v in
                ((n, getattr(self, n)) for n, _ in self._fields_)}


EXPORTED = {
    # name: (restype, argtypes)
    "sahara_gpu_last_error": (C.c_char_p, []),
    "sahara_build_id": (C.c_char_p, []),
    "sahara_gpu_device_count": (C.c_int, []),
    "sahara_gpu_open": (C.c_int, [C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "sahara_gpu_open_file": (C.c_int, [C.c_int, C.c_char_p, C.POINTER(C.c_void_p)]),
    "sahara_gpu_build": (C.c_int, [C.c_int, u8p, u64p, C.c_uint64, C.c_uint32, C.c_uint32,
                                   C.POINTER(C.c_void_p)]),
    "sahara_gpu_save": (C.c_int, [C.c_void_p, C.c_char_p]),
    "sahara_gpu_index_info": (C.c_int, [C.c_void_p, C.POINTER(IndexInfo)]),
    "sahara_gpu_export": (C.c_int, [C.c_void_p, u8p, u8p, u64p, u32p, u64p, u64p]),
    "sahara_gpu_export_sa": (C.c_int, [C.c_void_p, u32p]),
    "sahara_gpu_export_text": (C.c_int, [C.c_void_p, u8p]),
    "sahara_gpu_set_mode": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "sahara_gpu_select_part": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sahara_gpu_part_info": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "sahara_gpu_search": (C.c_int, [C.c_void_p, u8p, C.c_uint64, C.c_uint32, u32p, u32p, u32p,
                                    C.c_uint32, C.c_int, C.c_uint32, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_uint64)]),
    "sahara_gpu_search_reads": (C.c_int, [C.c_void_p, u8p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64, u32p, u32p,
                                          u32p, C.c_uint32, C.c_int, C.c_uint32, C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_uint64)]),
    "sahara_gpu_search_reads_compact": (C.c_int, [C.c_void_p, u8p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64,
                                                  u32p, u32p, u32p, C.c_uint32, C.c_int, C.POINTER(HitBlocks)]),
    "sahara_gpu_free_blocks": (None, [C.POINTER(HitBlocks)]),
    "sahara_gpu_search_packed": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u64p, C.c_uint64, C.c_uint64, C.c_uint32,
                                           C.c_int, C.c_uint64, u32p, u32p, u32p, C.c_uint32, C.c_int, C.c_uint32,
                                           C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "sahara_gpu_prepare": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32]),
    "sahara_gpu_search_packed_compact": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u64p, C.c_uint64, C.c_uint64,
                                                   C.c_uint32, C.c_int, C.c_uint64, u32p, u32p, u32p, C.c_uint32,
                                                   C.c_int, C.POINTER(HitBlocks)]),
    "sahara_read_fasta": (C.c_int, [C.c_char_p, C.c_uint32, C.c_int, C.c_uint32, C.POINTER(FastaOut)]),
    "sahara_free_fasta": (None, [C.POINTER(FastaOut)]),
    "sahara_host_alloc": (C.c_void_p, [C.c_size_t]),
    "sahara_host_free": (None, [C.c_void_p]),
    "sahara_gpu_search_best": (C.c_int, [C.c_void_p, u8p, C.c_uint64, C.c_uint32, u32p, u32p, u32p,
                                         u32p, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_uint64)]),
    "sahara_gpu_stage": (C.c_int, [C.c_void_p, u8p, C.c_uint64, C.c_uint32, u32p, u32p, u32p,
                                   C.c_uint32, C.c_int]),
    "sahara_gpu_run": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)]),
    "sahara_gpu_fetch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "sahara_gpu_digest": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "sahara_gpu_copy_hits": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]),
    "sahara_gpu_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "sahara_gpu_placement": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "sahara_gpu_free": (None, [C.c_void_p]),
    "sahara_gpu_close": (None, [C.c_void_p]),
    "sahara_scheme_generators": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int]),
    "sahara_scheme": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_int, u32p, u32p, u32p,
                                C.c_int]),
    "sahara_scheme_dynamic": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                        C.c_double, u32p, C.c_int, u32p, u32p, u32p, C.c_int]),
    "sahara_scheme_parts": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int),
                                      C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                      C.c_int]),
    "sahara_scheme_counts": (C.c_int, [u32p, u32p, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                       C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "sahara_synth_reference": (C.c_int, [C.c_uint64, C.c_uint32, u64p, C.c_uint64, u8p]),
    "sahara_synth_reads": (C.c_int, [u8p, u64p, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32,
                                     C.c_uint32, C.c_uint64, u8p, u64p]),
    "sahara_synth_reads_typed": (C.c_int, [u8p, u64p, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32,
                                           C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, u8p, u64p]),
    "sahara_interleave_rc": (C.c_int, [u8p, C.c_uint64, C.c_uint32, C.c_uint32, u8p]),
    "sahara_pack_2bit": (C.c_int, [u8p, C.c_uint64, C.c_uint32, C.c_int, u8p, u32p, C.c_uint64,
                                   C.POINTER(C.c_uint64)]),
}


def library_path():
    # SAHARA_HIP_LIB: another build of the same library (A/B benchmarks)
    return os.environ.get("SAHARA_HIP_LIB") or os.path.join(_HERE, "lib", "libsahara_hip.so")


def lib():
    """Load libsahara_hip.so. Raises if it is missing: there is no fallback."""
    global _LIB
    if _LIB is None:
        path = library_path()
        if not os.path.exists(path):
            raise ImportError(f"sahara_amd HIP extension missing: {path} (run `make` / "
                              f"__graft_entry__.build())")
        L = C.CDLL(path)
        for name, (res, args) in EXPORTED.items():
            if os.environ.get("SAHARA_HIP_LIB") and not hasattr(L, name):
                continue  # an older build under A/B comparison
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def build_id():
    """The library's build id (sahara_build_id: SHA-256 prefix of its sources, tools/build_id.py);
    "unknown" for an older build loaded through SAHARA_HIP_LIB (A/B runs)."""
    f = getattr(lib(), "sahara_build_id", None)
    return f().decode() if f else "unknown"


def _check(rc):
    if rc != 0:
        msg = lib().sahara_gpu_last_error()
        raise SaharaError(msg.decode() if msg else f"error {rc}")


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


def _records_to_flat(records):
    recs = [np.ascontiguousarray(r, dtype=np.uint8) for r in records]
    if not recs:
        raise SaharaError("reference is empty")
    flat = np.ascontiguousarray(np.concatenate(recs))
    lens = np.array([len(r) for r in recs], dtype=np.uint64)
    return flat, lens


class BiFMIndex:
    """GPU-resident bidirectional FM-index (fmc::BiFMIndex<Sigma, InterleavedBitvector16>)."""

    def __init__(self, handle, device):
        self._h = C.c_void_p(handle)
        self.device = device

    @classmethod
    def build(cls, records, sigma=6, sampling_rate=16, device=0):
        flat, lens = _records_to_flat(records)
        h = C.c_void_p()
        _check(lib().sahara_gpu_build(device, _p(flat, u8p), _p(lens, u64p), len(lens), sigma,
                                      sampling_rate, C.byref(h)))
        return cls(h.value, device)

    @classmethod
    def build_flat(cls, flat, rec_lens, sigma=6, sampling_rate=16, device=0):
        flat = np.ascontiguousarray(flat, dtype=np.uint8)
        lens = np.ascontiguousarray(rec_lens, dtype=np.uint64)
        h = C.c_void_p()
        _check(lib().sahara_gpu_build(device, _p(flat, u8p), _p(lens, u64p), len(lens), sigma,
                                      sampling_rate, C.byref(h)))
        return cls(h.value, device)

    @classmethod
    def load(cls, path, device=0):
        h = C.c_void_p()
        _check(lib().sahara_gpu_open_file(device, str(path).encode(), C.byref(h)))
        return cls(h.value, device)

    @classmethod
    def from_bytes(cls, data, device=0):
        buf = np.frombuffer(data, dtype=np.uint8)
        h = C.c_void_p()
        _check(lib().sahara_gpu_open(device, buf.ctypes.data_as(C.c_void_p), buf.nbytes, C.byref(h)))
        return cls(h.value, device)

    def save(self, path):
        _check(lib().sahara_gpu_save(self._h, str(path).encode()))

    def info(self):
        i = IndexInfo()
        _check(lib().sahara_gpu_index_info(self._h, C.byref(i)))
        return {n: getattr(i, n) for n, _ in i._fields_}

    @property
    def sigma(self):
        return self.info()["sigma"]

    def export(self):
        inf = self.part_info()
        n = inf["n"]
        bf = np.zeros(n, np.uint8)
        br = np.zeros(n, np.uint8)
        sb = np.zeros(n // 64 + 1, np.uint64)
        smp = np.zeros(max(inf["n_samples"], 1), np.uint32)
        Cc = np.zeros(8, np.uint64)
        rl = np.zeros(max(inf["n_records"], 1), np.uint64)
        _check(lib().sahara_gpu_export(self._h, _p(bf, u8p), _p(br, u8p), _p(sb, u64p),
                                       _p(smp, u32p), _p(Cc, u64p), _p(rl, u64p)))
        return dict(bwt_f=bf, bwt_r=br, sampled=sb, samples=smp[: inf["n_samples"]],
                    C=Cc[: inf["sigma"] + 1], rec_lens=rl[: inf["n_records"]], n=n,
                    sigma=inf["sigma"], rate=inf["sampling_rate"])

    def export_sa(self):
        n = self.part_info()["n"]
        sa = np.zeros(n, np.uint32)
        _check(lib().sahara_gpu_export_sa(self._h, _p(sa, u32p)))
        return sa

    def export_text(self):
        n = self.part_info()["n"]
        t = np.zeros(n, np.uint8)
        _check(lib().sahara_gpu_export_text(self._h, _p(t, u8p)))
        return t

    def select_part(self, part):
        """Multi-part index: which part export() / export_sa() / export_text() read."""
        _check(lib().sahara_gpu_select_part(self._h, part))
        self._part = part

    def part_info(self, part=None):
        i = IndexInfo()
        _check(lib().sahara_gpu_part_info(self._h, getattr(self, "_part", 0) if part is None else part, C.byref(i)))
        return {n: getattr(i, n) for n, _ in i._fields_}

    def set_mode(self, verify=True, locate_sa=True):
        """verify: continue singleton intervals against the resident text;
        locate_sa: locate through the resident full SA (else LF walks)."""
        _check(lib().sahara_gpu_set_mode(self._h, int(verify), int(locate_sa)))

    # ---- device-resident path (bench) ----
    def stage(self, queries, scheme, edit=True):
        q = np.ascontiguousarray(queries, dtype=np.uint8)
        pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
        _check(lib().sahara_gpu_stage(self._h, _p(q, u8p), q.shape[0], q.shape[1], _p(pi, u32p),
                                      _p(l, u32p), _p(u, u32p), pi.shape[0], int(edit)))

    def run(self, count=False):
        n = C.c_uint64()
        _check(lib().sahara_gpu_run(self._h, int(count), C.byref(n)))
        return n.value

    def fetch(self):
        n = C.c_uint64()
        st = self.stats()
        out = np.zeros(max(st["hits"], 1), HIT_DTYPE)
        _check(lib().sahara_gpu_fetch(self._h, out.ctypes.data_as(C.c_void_p), len(out), C.byref(n)))
        return out[: n.value]

    def copy_hits(self, dst_ptr, capacity, qid_offset=0):
        """Copy the last run's hits (HIT_DTYPE records) into device memory at
        dst_ptr (e.g. a torch tensor's data_ptr() on this GPU), qids shifted by
        qid_offset. Returns the number of records."""
        n = C.c_uint64()
        _check(lib().sahara_gpu_copy_hits(self._h, C.c_void_p(dst_ptr), capacity, qid_offset, C.byref(n)))
        return n.value

    def digest(self):
        d = C.c_uint64()
        _check(lib().sahara_gpu_digest(self._h, C.byref(d)))
        return d.value

    def placement(self):
        """(HIP device, NUMA node or -1, CPUs the context's threads are bound to)."""
        d, node, ncpu = C.c_int(), C.c_int(), C.c_int()
        _check(lib().sahara_gpu_placement(self._h, C.byref(d), C.byref(node), C.byref(ncpu)))
        return {"device": d.value, "numa_node": node.value, "n_cpus": ncpu.value}

    def prepare(self, n_patterns, length=0):
        """sahara_gpu_prepare: the first search call's one-time work ahead
        (pinned hit sink, device buffers of the streamed pass)."""
        _check(lib().sahara_gpu_prepare(self._h, int(n_patterns), int(length)))

    def stats(self):
        s = Stats()
        _check(lib().sahara_gpu_stats(self._h, C.byref(s)))
        return s.as_dict()

    def close(self):
        if self._h and self._h.value:
            lib().sahara_gpu_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _HitBuffer:
    """Owner of a library-allocated hit array: the numpy view keeps it alive,
    and the buffer goes back to sahara_gpu_free with the last reference."""

    def __init__(self, ptr, n):
        self.ptr = ptr
        self.__array_interface__ = {"shape": (n,), "typestr": "|V%d" % HIT_DTYPE.itemsize,
                                    "descr": HIT_DTYPE.descr, "data": (ptr, False), "version": 3}

    def __del__(self):
        if self.ptr:
            lib().sahara_gpu_free(C.c_void_p(self.ptr))
            self.ptr = None


def _hits_array(out, n):
    if not out.value:
        return np.zeros(0, HIT_DTYPE)
    if n == 0:
        lib().sahara_gpu_free(out)
        return np.zeros(0, HIT_DTYPE)
    a = np.asarray(_HitBuffer(out.value, n))  # zero-copy; the base frees the buffer
    return a.view(HIT_DTYPE)


def search(index, queries, scheme, edit=True, max_hits=0):
    """fmc::search_ng24::search<Edit> + fmc::LocateLinear (search.cpp:218-250).

    queries: (n_patterns, len) uint8 ranks (qid = row); scheme: (pi, l, u),
    each (n_searches, len). Returns a HIT_DTYPE array sorted by
    (qid, seq_id, pos, err)."""
    q = np.ascontiguousarray(queries, dtype=np.uint8)
    if q.ndim != 2 or q.shape[0] == 0:
        raise SaharaError("queries must be a non-empty (n_patterns, len) array")
    pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
    out = C.c_void_p()
    n = C.c_uint64()
    _check(lib().sahara_gpu_search(index._h, _p(q, u8p), q.shape[0], q.shape[1], _p(pi, u32p),
                                   _p(l, u32p), _p(u, u32p), pi.shape[0], int(edit), max_hits,
                                   C.byref(out), C.byref(n)))
    return _hits_array(out, n.value)


def search_reads(index, reads, scheme, edit=True, reverse=True, limit=0, max_hits=0):
    """Query ingest + search + locate in one call (search.cpp:111-127, 218-250):
    the reverse complements are interleaved on the device (qid 2i = read i,
    2i + 1 = its reverse complement; reverse=False: qid i = read i), and
    limit > 0 cuts the query list after the interleave (--limit_queries).
    Returns the same sorted HIT_DTYPE array as search() over the interleaved
    patterns."""
    r = np.ascontiguousarray(reads, dtype=np.uint8)
    if r.ndim != 2 or r.shape[0] == 0:
        raise SaharaError("reads must be a non-empty (n_reads, len) array")
    pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
    out = C.c_void_p()
    n = C.c_uint64()
    _check(lib().sahara_gpu_search_reads(index._h, _p(r, u8p), r.shape[0], r.shape[1], int(reverse), int(limit),
                                         _p(pi, u32p), _p(l, u32p), _p(u, u32p), pi.shape[0], int(edit), max_hits,
                                         C.byref(out), C.byref(n)))
    return _hits_array(out, n.value)


class _Blocks:
    """Owner of one sahara_hit_blocks: frees it when released or when the last
    reference goes (the CompactHits, or an array made over its records)."""

    def __init__(self, blocks):
        self.b = blocks

    def free(self):
        if self.b is not None:
            lib().sahara_gpu_free_blocks(C.byref(self.b))
            self.b = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class _OwnedRecords:
    """numpy array interface over the records of a _Blocks that keeps it
    alive: an array made from it (CompactHits.recs, and every view of that)
    holds the owner, so the memory cannot go back to the library's pool while
    any of them exists. (The owner is not the CompactHits itself: no cycle,
    so a dropped result frees its memory at once.)"""

    def __init__(self, owner, addr, n):
        self._owner = owner
        self.__array_interface__ = {"shape": (n,), "typestr": "<u8", "data": (addr, True), "version": 3}


class CompactHits:
    """Hits of sahara_gpu_search_reads_compact (include/sahara_hip.h
    sahara_hit_blocks): 8-B records in page-locked host memory, one block per
    batch. `recs` is a read-only zero-copy view that keeps the memory alive;
    close() drops this object's hold on it: the memory goes back to the
    library's pool at once, unless a view of `recs` taken earlier is still
    alive, which keeps it until that view goes. to_hits() expands the records
    to HIT_DTYPE."""

    def __init__(self, blocks, index):
        self._own = _Blocks(blocks)
        self._b = blocks
        self._index = index  # rec_starts belongs to the context
        n = blocks.n_hits
        if n:
            addr = C.cast(blocks.recs, C.c_void_p).value
            self.recs = np.asarray(_OwnedRecords(self._own, addr, n))
        else:
            self.recs = np.zeros(0, np.uint64)
        nb = blocks.n_blocks
        self.block_qid0 = np.ctypeslib.as_array(blocks.block_qid0, shape=(nb,)).copy() if nb else np.zeros(0, np.uint64)
        self.block_end = np.ctypeslib.as_array(blocks.block_end, shape=(nb,)).copy() if nb else np.zeros(0, np.uint64)
        self.rec_starts = np.ctypeslib.as_array(blocks.rec_starts, shape=(blocks.n_records + 1,)).copy()

    def __len__(self):
        return int(self._b.n_hits) if self._b is not None else 0

    def to_hits(self):
        n = len(self)
        out = np.zeros(n, HIT_DTYPE)
        if n == 0:
            return out
        v = self.recs
        counts = np.diff(np.concatenate([[0], self.block_end])).astype(np.int64)
        base = np.repeat(self.block_qid0, counts)
        out["qid"] = base + (v >> np.uint64(36))
        g = (v >> np.uint64(4)) & np.uint64(0xFFFFFFFF)
        seq = np.searchsorted(self.rec_starts, g, side="right") - 1
        out["seq_id"] = seq
        out["pos"] = g - self.rec_starts[seq]
        out["err"] = (v & np.uint64(15)).astype(np.uint32)
        return out

    def close(self):
        if self._b is not None:
            self.recs = None
            self._own = None  # freed with the last reference (this one, or a view's)
            self._b = None


def search_reads_compact(index, reads, scheme, edit=True, reverse=True, limit=0):
    """search_reads (max_hits = 0) with the hits as compact 8-B records written
    by the device into pinned host memory (sahara_gpu_search_reads_compact)."""
    r = np.ascontiguousarray(reads, dtype=np.uint8)
    if r.ndim != 2 or r.shape[0] == 0:
        raise SaharaError("reads must be a non-empty (n_reads, len) array")
    pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
    b = HitBlocks()
    _check(lib().sahara_gpu_search_reads_compact(index._h, _p(r, u8p), r.shape[0], r.shape[1], int(reverse),
                                                 int(limit), _p(pi, u32p), _p(l, u32p), _p(u, u32p), pi.shape[0],
                                                 int(edit), C.byref(b)))
    return CompactHits(b, index)


class PackedReads:
    """Reads two bits per symbol, the form sahara_gpu_search_packed[_compact]
    take and `sahara search`'s FASTA ingest produces (read_fasta(form=2)):
    `codes` holds stream symbol s at bits 2 (s % 4) of byte s / 4 (A C G T =
    0 1 2 3), read i is symbols [sym0 + i * length, sym0 + (i + 1) * length),
    and `n_pos` lists the stream positions of N (dna5), ascending."""

    def __init__(self, codes, n_reads, length, n_pos=None, sym0=0):
        self.codes = np.ascontiguousarray(codes, dtype=np.uint8)
        self.n_reads, self.length, self.sym0 = int(n_reads), int(length), int(sym0)
        self.n_pos = np.ascontiguousarray(n_pos if n_pos is not None else np.zeros(0), dtype=np.uint64)
        if self.codes.size * 4 < self.sym0 + self.n_reads * self.length:
            raise SaharaError("packed codes shorter than the reads they should hold")

    def shard(self, r0, r1):
        """Reads [r0, r1) over the same buffers (a shard of the stream)."""
        return PackedReads(self.codes, r1 - r0, self.length, self.n_pos, self.sym0 + r0 * self.length)


class _Pinned:
    """Owner of page-locked host memory (sahara_host_alloc), freed with the
    last array over it."""

    def __init__(self, nbytes):
        self.p = lib().sahara_host_alloc(max(1, nbytes))
        if not self.p:
            raise SaharaError(lib().sahara_gpu_last_error().decode())
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.p, False), "version": 3}

    def __del__(self):
        try:
            lib().sahara_host_free(self.p)
        except Exception:
            pass


def host_array(nbytes):
    """uint8 array of nbytes in page-locked host memory (sahara_host_alloc):
    the packed search calls DMA reads kept there without copying them."""
    return np.asarray(_Pinned(int(nbytes)))


def pack_reads(reads, sigma=6, pinned=False):
    """(n_reads, len) ranks -> PackedReads (the library's host packer,
    sahara_pack_2bit; raises on a byte that is no rank of the alphabet);
    pinned: the codes in page-locked memory (host_array)."""
    r = np.ascontiguousarray(reads, dtype=np.uint8)
    codes, pos, bad = pack_2bit(r, sigma, out=host_array((r.size + 3) // 4) if pinned else None)
    if bad:
        raise SaharaError("reads hold a byte that is no rank of the alphabet")
    return PackedReads(codes, r.shape[0], r.shape[1], pos.astype(np.uint64))


def _packed_args(packed, scheme):
    pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
    if packed.n_reads <= 0:
        raise SaharaError("no reads")
    return (_p(packed.codes, u8p), packed.sym0, _p(packed.n_pos, u64p) if packed.n_pos.size else None,
            packed.n_pos.size, packed.n_reads, packed.length), (pi, l, u)


def search_packed(index, packed, scheme, edit=True, reverse=True, limit=0, max_hits=0):
    """search_reads from PackedReads (sahara_gpu_search_packed)."""
    a, (pi, l, u) = _packed_args(packed, scheme)
    out = C.c_void_p()
    n = C.c_uint64()
    _check(lib().sahara_gpu_search_packed(index._h, *a, int(reverse), int(limit), _p(pi, u32p), _p(l, u32p),
                                          _p(u, u32p), pi.shape[0], int(edit), max_hits, C.byref(out), C.byref(n)))
    return _hits_array(out, n.value)


def search_packed_compact(index, packed, scheme, edit=True, reverse=True, limit=0):
    """search_reads_compact from PackedReads (sahara_gpu_search_packed_compact):
    `sahara search`'s call at the drop-in boundary."""
    a, (pi, l, u) = _packed_args(packed, scheme)
    b = HitBlocks()
    _check(lib().sahara_gpu_search_packed_compact(index._h, *a, int(reverse), int(limit), _p(pi, u32p), _p(l, u32p),
                                                  _p(u, u32p), pi.shape[0], int(edit), C.byref(b)))
    return CompactHits(b, index)


def read_fasta(path, sigma=6, form=1, threads=0):
    """The library's FASTA ingest (sahara_read_fasta; search.cpp:111-130):
    dict with `data` (form 1: one rank per symbol, 255 = invalid; form 2: two
    bits per symbol), `offs` (record i = symbols [offs[i], offs[i+1])),
    `n_pos` (form 2: N positions) and `bad` (None, or (record, position,
    character, header) of the first invalid character)."""
    own = _FastaOwner()
    f = own.f
    _check(lib().sahara_read_fasta(os.fsencode(path), sigma, form, threads, C.byref(f)))
    nb = f.n_symbols if form == 1 else (f.n_symbols + 3) // 4
    # form 2: a zero-copy view of the library's page-locked buffer (kept alive
    # by the array); form 1 and the small arrays: copies
    if nb and form == 2:
        data = np.asarray(_FastaData(own, C.cast(f.data, C.c_void_p).value, nb))
    else:
        data = np.ctypeslib.as_array(f.data, shape=(nb,)).copy() if nb else np.zeros(0, np.uint8)
    offs = np.ctypeslib.as_array(f.offs, shape=(f.n_records + 1,)).copy() if f.n_records else np.zeros(0, np.uint64)
    npos = np.ctypeslib.as_array(f.n_pos, shape=(f.n_count,)).copy() if f.n_count else np.zeros(0, np.uint64)
    bad = (int(f.bad_record), int(f.bad_pos), chr(f.bad_char), f.bad_id.decode()) if f.bad else None
    return {"data": data, "offs": offs, "n_pos": npos, "n_symbols": int(f.n_symbols), "bad": bad}


class _FastaOwner:
    def __init__(self):
        self.f = FastaOut()

    def __del__(self):
        try:
            lib().sahara_free_fasta(C.byref(self.f))
        except Exception:
            pass


class _FastaData:
    def __init__(self, owner, addr, n):
        self._owner = owner
        self.__array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (addr, False), "version": 3}


def search_best(index, queries, schemes, max_hits=0):
    """fmc::search_ng21::search_best[_n] + LocateLinear (search.cpp:233-250).

    schemes: list of (pi, l, u), entry j being the expanded exact-j scheme
    (generator(j, j) expanded to len, search.cpp:235-237). Each query gets the
    hits of the smallest j that reports any. Sorted HIT_DTYPE array."""
    q = np.ascontiguousarray(queries, dtype=np.uint8)
    if q.ndim != 2 or q.shape[0] == 0:
        raise SaharaError("queries must be a non-empty (n_patterns, len) array")
    def cat(i):
        parts = [np.asarray(s[i], np.uint32).ravel() for s in schemes] or [np.zeros(1, np.uint32)]
        return np.ascontiguousarray(np.concatenate(parts))
    pi, l, u = cat(0), cat(1), cat(2)
    ns = np.array([len(s[0]) for s in schemes], np.uint32)
    out = C.c_void_p()
    n = C.c_uint64()
    _check(lib().sahara_gpu_search_best(index._h, _p(q, u8p), q.shape[0], q.shape[1], _p(pi, u32p),
                                        _p(l, u32p), _p(u, u32p), _p(ns, u32p), len(schemes), max_hits,
                                        C.byref(out), C.byref(n)))
    return _hits_array(out, n.value)


def scheme_generators():
    n = lib().sahara_scheme_generators(None, None, 0)
    names = (C.c_char_p * n)()
    descs = (C.c_char_p * n)()
    lib().sahara_scheme_generators(names, descs, n)
    return {names[i].decode(): descs[i].decode() for i in range(n)}


def search_scheme(generator, min_k, max_k, length, hamming=False):
    """generator::all[name](minK, maxK) -> expand(len) [-> limitToHamming] (search.cpp:186-212, :226)."""
    L = lib()
    n = L.sahara_scheme(generator.encode(), min_k, max_k, length, int(hamming), None, None, None, 0)
    if n < 0:
        names = ", ".join(scheme_generators())
        raise SaharaError(f'unknown search scheme generetaror "{generator}", valid generators are: {names}')
    pi = np.zeros((n, length), np.uint32)
    l = np.zeros((n, length), np.uint32)
    u = np.zeros((n, length), np.uint32)
    rc = L.sahara_scheme(generator.encode(), min_k, max_k, length, int(hamming), _p(pi, u32p),
                         _p(l, u32p), _p(u, u32p), n)
    if rc != n:
        raise SaharaError(f"cannot expand scheme {generator} to length {length} (rc={rc})")
    return pi, l, u


def search_scheme_dynamic(generator, min_k, max_k, length, hamming=False, edit=True, sigma=6, text_len=3e9):
    """--dynamic_generator: expanded scheme with WNC-optimised part sizes -> ((pi, l, u), sizes)."""
    L = lib()
    n = L.sahara_scheme_dynamic(generator.encode(), min_k, max_k, length, int(hamming), int(edit), sigma,
                                float(text_len), None, 0, None, None, None, 0)
    if n < 0:
        raise SaharaError(f"unknown search scheme generator {generator!r}")
    sizes = np.zeros(64, np.uint32)
    pi = np.zeros((n, length), np.uint32)
    l = np.zeros((n, length), np.uint32)
    u = np.zeros((n, length), np.uint32)
    rc = L.sahara_scheme_dynamic(generator.encode(), min_k, max_k, length, int(hamming), int(edit), sigma,
                                 float(text_len), _p(sizes, u32p), 64, _p(pi, u32p), _p(l, u32p), _p(u, u32p), n)
    if rc != n:
        raise SaharaError(f"cannot expand scheme {generator} to length {length} (rc={rc})")
    P = scheme_parts(generator, min_k, max_k)[0].shape[1]
    return (pi, l, u), sizes[:P].copy()


def scheme_parts(generator, min_k, max_k):
    P = C.c_int()
    n = lib().sahara_scheme_parts(generator.encode(), min_k, max_k, C.byref(P), None, None, None, 0)
    if n < 0:
        raise SaharaError(f"unknown generator {generator}")
    cap = n * P.value
    pi = (C.c_int * cap)()
    l = (C.c_int * cap)()
    u = (C.c_int * cap)()
    lib().sahara_scheme_parts(generator.encode(), min_k, max_k, C.byref(P), pi, l, u, cap)
    sh = (n, P.value)
    return (np.array(pi[:], np.int64).reshape(sh), np.array(l[:], np.int64).reshape(sh),
            np.array(u[:], np.int64).reshape(sh))


def scheme_counts(scheme, edit, sigma, text_len):
    pi, l, u = (np.ascontiguousarray(a, dtype=np.uint32) for a in scheme)
    a, b = C.c_double(), C.c_double()
    lib().sahara_scheme_counts(_p(l, u32p), _p(u, u32p), pi.shape[0], pi.shape[1], int(edit), sigma,
                               float(text_len), C.byref(a), C.byref(b))
    return a.value, b.value


def synth_reference(lengths, sigma=6, seed=42):
    lens = np.ascontiguousarray(lengths, dtype=np.uint64)
    out = np.zeros(int(lens.sum()), np.uint8)
    _check(lib().sahara_synth_reference(seed, sigma, _p(lens, u64p), len(lens), _p(out, u8p)))
    return out, lens


def synth_reads(flat, rec_lens, n_reads, length, errors, sigma=6, seed=7, with_origin=False, substitutions=0,
                insertions=0, deletions=0):
    """Reads with `errors` transcript errors of uniform type S/I/D, plus fixed numbers of each type
    (read_simulator.cpp semantics)."""
    flat = np.ascontiguousarray(flat, dtype=np.uint8)
    lens = np.ascontiguousarray(rec_lens, dtype=np.uint64)
    out = np.zeros((n_reads, length), np.uint8)
    origin = np.zeros((n_reads, 2), np.uint64) if with_origin else None
    _check(lib().sahara_synth_reads_typed(_p(flat, u8p), _p(lens, u64p), len(lens), sigma, n_reads, length,
                                          substitutions, insertions, deletions, errors, seed, _p(out, u8p),
                                          _p(origin, u64p)))
    return (out, origin) if with_origin else out


def pack_2bit(ranks, sigma=6, scalar=False, out=None):
    """Host half of the streamed upload at two bits per symbol (staging.cpp
    pack2Avx512 / pack2Avx2 / pack2Scalar): (packed bytes, N positions,
    bad-rank flag). scalar: False = widest SIMD, True = scalar, 2 = AVX2 at most.
    out: a uint8 array of (n + 3) // 4 bytes to pack into."""
    r = np.ascontiguousarray(ranks, dtype=np.uint8).ravel()
    if out is None:
        out = np.zeros((r.size + 3) // 4, np.uint8)
    assert out.dtype == np.uint8 and out.size == (r.size + 3) // 4 and out.flags.c_contiguous
    cnt = C.c_uint64(0)
    rc = lib().sahara_pack_2bit(_p(r, u8p), r.size, sigma, int(scalar), _p(out, u8p), None, 0, C.byref(cnt))
    if rc < 0:
        _check(rc)
    pos = np.zeros(max(1, cnt.value), np.uint32)
    lib().sahara_pack_2bit(_p(r, u8p), r.size, sigma, int(scalar), _p(out, u8p), _p(pos, u32p), pos.size,
                           C.byref(cnt))
    return out, pos[:cnt.value], bool(rc)


def interleave_rc(reads, sigma=6):
    """search.cpp:121-123: qid 2i = read i, 2i+1 = its reverse complement."""
    r = np.ascontiguousarray(reads, dtype=np.uint8)
    out = np.zeros((2 * r.shape[0], r.shape[1]), np.uint8)
    _check(lib().sahara_interleave_rc(_p(r, u8p), r.shape[0], r.shape[1], sigma, _p(out, u8p)))
    return out


def load_fasta(path, sigma=6):
    """Minimal FASTA reader -> list of (id, ranks) (ivio::fasta::reader + convert_char_to_rank)."""
    table = np.full(256, 255, np.uint8)
    chars = DNA5["chars"] if sigma == 6 else DNA4["chars"]
    for r, ch in enumerate(chars):
        if r == 0:
            continue
        table[ord(ch)] = r
        table[ord(ch.lower())] = r
    recs, name, seq = [], None, []
    with open(path, "rb") as f:
        for line in f:
            line = line.rstrip(b"\r\n")
            if line.startswith(b">"):
                if name is not None:
                    recs.append((name, table[np.frombuffer(b"".join(seq), np.uint8)]))
                name, seq = line[1:].decode(), []
            elif line:
                seq.append(line)
    if name is not None:
        recs.append((name, table[np.frombuffer(b"".join(seq), np.uint8)]))
    return recs
