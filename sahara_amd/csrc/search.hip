// search.hip — search-scheme DFS + locate on the GPU-resident FM-index (gfx950).
//
// Replaces fmc::search_ng24::search<Edit> (/root/reference/src/sahara/search.cpp:227,230)
// and fmc::LocateLinear (search.cpp:244-250) — semantics policy P0,
// docs/semantics.md; CPU restatement in oracle/oracle.cpp (Searcher::visit).
//
// Two phases per batch of patterns, both "one lane = one depth-first search,
// the wave shares a work queue":
//
// Phase 1, kSearchFM: work items are (pattern, search) pairs. Each node ranks
// all sigma-1 symbols at lo and lo+len on the BWT of its extension side — one
// 64-B Occ line per distinct 64-row block. Lanes of a pair fetch each other's
// lines together (<= 32 distinct lines per load instruction: address
// translation stays off the critical path on a multi-GB index, see
// tools/gather_bench.hip) and swap halves with DPP. As soon as a node's
// interval holds at most `split` rows, the node is handed to phase 2 as one
// *text task* per row instead of being ranked further.
//
// Phase 2, kSearchTextBatch: a text task is a node whose string t has a single
// occurrence. Extending it by symbol c is non-empty iff c is the text's own
// next symbol, so the rest of its subtree is the same DFS run against the
// text. The lane copies the window of the 4-bit text that the subtree can
// reach (full SA: one read) and the packed pattern into LDS and expands the
// subtree there, without touching HBM. Nodes whose remaining positions admit
// no further error are decided by one comparison of the remaining pattern
// against the window.
//
// Both DFSs push the match child first and the error children above it and
// continue with one error child in registers, so a stack holds at most the
// siblings of the error edges on the current path: <= k*(2*sigma-2) (FM) or
// <= 2k (text) entries, independent of the pattern length.
//
// The multiset of (qid, text position, e) leaves equals the reference DFS's:
// a node of interval [lb, lb+len) expands to the same (path, occurrence)
// pairs whether it is ranked or split into its len occurrences.
//
// Leaves are compacted into the hit buffer with a wave ballot + prefix count
// into per-wave reserved slot ranges (one atomic per 64 slots). Overflow of
// any buffer is flagged; the host re-runs the batch with a larger buffer.
//
// Locate: FM leaves resolve rows through the resident full SA (one read per
// row) or, in the reference mode, by LF walks to the SA samples, straight
// into per-query segments (counting sort by qid: row counts, exclusive scan).
// Keys text position << 4 | e are then sorted within each segment — in
// registers for the usual <= 8 rows, by a segmented radix sort for longer
// segments — for the canonical (qid, seq_id, pos, e) order.

#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#include "search.h"

namespace sahara {
namespace {

// Pointers that come from memory (the slot table), from integers (Occ line
// addresses) or that may point to LDS or global memory (a stack level) are
// generic: accesses through them are flat instructions, which also count
// against the LDS counter and make every LDS wait wait for them (and a flat
// access of LDS is slower than a ds_ one). Where they address global memory,
// say so. (The host pass of this file parses kernel bodies too, where class
// types in an address space do not convert: there the cast is a plain one.)
#if defined(__HIP_DEVICE_COMPILE__)
#define GLOB(T, p) ((__attribute__((address_space(1))) T*)(p))
#else
#define GLOB(T, p) ((T*)(p))
#endif
// A 16-B record through a global pointer: uint4 is a class type whose copy
// goes through a generic reference (a flat access again), a native vector is not
typedef uint32_t U32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 loadGlobal4(const uint4* p) {
    const U32x4 v = *GLOB(const U32x4, p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Swap a dword with the neighbour lane of the pair (DPP quad_perm [1,0,3,2]).
__device__ __forceinline__ uint32_t pairSwap(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}
__device__ __forceinline__ uint4 pairSwap4(const uint4& v) {
    return make_uint4(pairSwap(v.x), pairSwap(v.y), pairSwap(v.z), pairSwap(v.w));
}
__device__ __forceinline__ uint64_t pairSwap64(uint64_t v) {
    return (uint64_t)pairSwap((uint32_t)v) | ((uint64_t)pairSwap((uint32_t)(v >> 32)) << 32);
}

// Pair-cooperative fetch of the rank part (bytes 0..47) of one 64-B Occ line
// per lane. Must be called by all 64 lanes (wave-uniform control flow):
// for the pair (E = even lane's line, O = odd lane's line) four loads run
//   #1 E bytes 0-15 | 16-31   #2 E bytes 32-47 | 48-63
//   #3 O bytes 0-15 | 16-31   #4 O bytes 32-47 | 48-63
// (even | odd lane), so each wave instruction touches <= 32 distinct lines;
// two DPP swaps then hand each lane the chunks of its own line.
__device__ __forceinline__ void fetchLinePair(uint64_t own, bool need, bool odd, uint32_t cnt[5], uint64_t p[3]) {
    const uint64_t other = pairSwap64(own);
    const bool otherNeed = pairSwap(need ? 1u : 0u) != 0u;
    const uint64_t addrE = odd ? other : own, addrO = odd ? own : other;
    const bool needE = odd ? otherNeed : need, needO = odd ? need : otherNeed;
    const uint32_t half = odd ? 16u : 0u;
    uint4 r1 = make_uint4(0, 0, 0, 0), r2 = r1, r3 = r1, r4 = r1;
    if (needE) {
        r1 = loadGlobal4(reinterpret_cast<const uint4*>(addrE + half));
        r2 = loadGlobal4(reinterpret_cast<const uint4*>(addrE + 32 + half));
    }
    if (needO) {
        r3 = loadGlobal4(reinterpret_cast<const uint4*>(addrO + half));
        r4 = loadGlobal4(reinterpret_cast<const uint4*>(addrO + 32 + half));
    }
    // even: r1 = E0, r2 = E2, r3 = O0, r4 = O2 ; odd: r1 = E1, r2 = E3, r3 = O1, r4 = O3
    const uint4 g1 = pairSwap4(odd ? r1 : r3);  // even <- E1, odd <- O0
    const uint4 g2 = pairSwap4(r4);             // odd <- O2 (even receives O3, unused)
    const uint4 c0 = odd ? g1 : r1;
    const uint4 c1 = odd ? r3 : g1;
    const uint4 c2 = odd ? g2 : r2;
    cnt[0] = c0.x; cnt[1] = c0.y; cnt[2] = c0.z; cnt[3] = c0.w; cnt[4] = c1.x;
    p[0] = (uint64_t)c1.z | ((uint64_t)c1.w << 32);
    p[1] = (uint64_t)c2.x | ((uint64_t)c2.y << 32);
    p[2] = (uint64_t)c2.z | ((uint64_t)c2.w << 32);
}

__device__ __forceinline__ uint32_t pick5(const uint32_t v[5], uint32_t i) {
    uint32_t r = v[0];
    r = i == 1 ? v[1] : r;
    r = i == 2 ? v[2] : r;
    r = i == 3 ? v[3] : r;
    r = i == 4 ? v[4] : r;
    return r;
}

__device__ __forceinline__ uint32_t nib(uint32_t word, uint32_t i) { return (word >> ((i & 7u) * 4u)) & 0xFu; }

constexpr uint32_t kSeedChunk = 64;   // seeds a wave takes per atomic
// text tasks a wave takes per atomic (<= 64; 64 / 32 / 16 measured 1088 / 1021 /
// 891M reads/s at C3, profiles/r05_task_chunk_ab.txt)
constexpr uint32_t kTaskChunk = 64;
static_assert(kTaskChunk >= 1 && kTaskChunk <= 64, "a chunk's records sit one per lane");
constexpr uint32_t kHitChunk = 64;    // hit / task slots a wave reserves per atomic

// Per-wave slot reservation for append-only outputs (hits, tasks): ballot +
// prefix count inside the wave's current range; a fresh range of kHitChunk
// slots costs one atomic. All lanes must call it (wave-uniform).
struct SlotRange {
    uint32_t next = 0, end = 0;
    __device__ __forceinline__ bool take(bool want, uint32_t lane, uint64_t ltMask, uint32_t* counter,
                                         uint32_t& slot) {
        const uint64_t m = __ballot(want);
        if (!m) return false;
        const uint32_t cnt = (uint32_t)__popcll(m);
        const uint32_t rank = (uint32_t)__popcll(m & ltMask);
        const uint32_t avail = end - next;
        uint32_t base = 0;
        if (cnt > avail) {
            if (lane == 0) base = atomicAdd(counter, kHitChunk);
            base = __shfl(base, 0);
        }
        slot = rank < avail ? next + rank : base + (rank - avail);
        if (cnt > avail) { next = base + (cnt - avail); end = base + kHitChunk; }
        else next += cnt;
        return true;
    }
    // unused tail of the last range: empty records (len 0) for the locate scan
    __device__ __forceinline__ void close(uint32_t lane, uint4* buf, uint32_t cap) {
        for (uint32_t i = next + lane; i < end; i += 64)
            if (i < cap) buf[i] = make_uint4(0u, 0u, 0u, 0u);
    }
};

// Work queue split into kStripes stripes with one counter each (128 B apart):
// a wave starts on the stripe of its XCD (blockIdx % 8) and moves on when it
// is drained. A single counter serialises at ~90 chunk grabs per microsecond
// device-wide; eight of them keep a chunk grab off the critical path.
constexpr uint32_t kStripes = 8;
constexpr uint32_t kStripeStride = 32;  // u32 between counters
struct StripedQueue {
    uint32_t* ctr;
    uint32_t n, stripe, tries = 0;
    __device__ StripedQueue(uint32_t* c, uint32_t total) : ctr(c), n(total), stripe(blockIdx.x % kStripes) {}
    // next chunk [b, e) of at most `chunk` items (wave-uniform); false when all stripes are drained
    __device__ bool next(uint32_t lane, uint32_t chunk, uint32_t& b, uint32_t& e) {
        while (tries < kStripes) {
            const uint32_t s0 = (uint32_t)((uint64_t)n * stripe / kStripes);
            const uint32_t s1 = (uint32_t)((uint64_t)n * (stripe + 1) / kStripes);
            uint32_t off = 0;
            if (lane == 0) off = s0 < s1 ? atomicAdd(ctr + stripe * kStripeStride, chunk) : 0xFFFFFFFFu;
            off = __shfl(off, 0);
            if (off != 0xFFFFFFFFu && off < s1 - s0) {
                b = s0 + off;
                e = min(b + chunk, s1);
                return true;
            }
            stripe = (stripe + 1) % kStripes;
            ++tries;
        }
        return false;
    }
};

// Children of one DFS node under policy P0 (docs/semantics.md), with the
// stack discipline described at the top. `occ[c]` says whether the child of
// symbol c exists; `mk(c, kind)` builds it. Returns whether a child is kept
// in registers (through `next`).
template <int SIGMA, typename Node, typename MkChild, typename Push>
__device__ __forceinline__ bool expandChildren(const uint32_t occ[SIGMA], uint32_t cq, bool matchOK, bool misOK,
                                               bool delOK, bool insOK, const Node& insChild, MkChild mk, Push push,
                                               Node& next) {
    uint32_t nErr = insOK ? 1u : 0u;
    bool hasM = false;
#pragma unroll
    for (int c = 1; c < SIGMA; ++c) {
        if (occ[c]) {
            if ((uint32_t)c == cq) hasM = matchOK;
            else nErr += misOK ? 1u : 0u;
            nErr += delOK ? 1u : 0u;
        }
    }
    bool kept = false;
    auto emit = [&](const Node& v) {
        if (!kept) { next = v; kept = true; }
        else push(v);
    };
    if (hasM && nErr) push(mk((int)cq, 0));  // match child below all its error siblings
    if (insOK) emit(insChild);
#pragma unroll
    for (int c = 1; c < SIGMA; ++c) {
        if (occ[c]) {
            if ((uint32_t)c != cq && misOK) emit(mk(c, 1));
            if (delOK) emit(mk(c, 2));
        }
    }
    if (!kept && hasM) { next = mk((int)cq, 0); kept = true; }
    return kept;
}

// kind: 0 = match (M), 1 = substitution (S), 2 = deletion (D), 3 = insertion (I)
__device__ __forceinline__ uint32_t childMeta(uint32_t pos, uint32_t e, uint32_t lastL, uint32_t lastR, bool right,
                                              uint32_t dl, uint32_t kind) {
    const uint32_t op = kind == 2 ? OP_D : (kind == 3 ? OP_I : OP_MS);
    const uint32_t npos = kind == 2 ? pos : pos + 1u;
    const uint32_t ne = kind == 0 ? e : e + 1u;
    const uint32_t nl = pos == 0 ? op : (right ? lastL : op);
    const uint32_t nr = pos == 0 ? op : (right ? op : lastR);
    const uint32_t nd = dl + (kind == 2 ? 1u : 0u) - (kind == 3 ? 1u : 0u);
    return npos | (ne << 16) | (nl << 20) | (nr << 22) | (nd << 25);
}

// ========================================================= seeds ====
// One thread per work item (pattern, search): its starting cursor. A search
// whose first kmerK steps admit no error starts at depth kmerK from the k-mer
// table (the DFS would reach the same node through kmerK forced matches);
// items whose k-mer does not occur end here. Every other item starts at the
// root. Surviving items are appended (wave ballot + one atomic per wave) to
// the seed list that kSearchFM consumes.
// The k-mer table index of item i's error-free first part, or ~0u when the
// item starts at the root (no table, no error-free first part, or an N in it).
template <int SIGMA>
__device__ __forceinline__ uint32_t seedCode(const SeedArgs& a, uint32_t i) {
    if (i >= a.nitems || !a.kmer) return ~0u;
    const uint32_t pid = i / a.nsearch, s = i - pid * a.nsearch;
    const uint32_t ks = a.kmerStart[s];
    if (ks == 0xFFFFFFFFu) return ~0u;
    const uint32_t* pw = a.pats + (size_t)pid * a.patWords + (ks >> 3);
    const uint32_t w0 = pw[0], w1 = pw[1], w2 = pw[2];
    const uint32_t sh = (ks & 7u) * 4u;
    const uint64_t run = (uint64_t)__builtin_amdgcn_alignbit(w1, w0, sh) |
                         ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sh) << 32);
    uint32_t code = 0;
    bool acgt = true;
    for (uint32_t j = 0; j < a.kmerK; ++j) {
        const uint32_t c = (uint32_t)(run >> (4u * j)) & 0xFu;  // A1 C2 G3 (N4) T5|T4
        acgt = acgt && !(SIGMA == 6 && c == 4u);
        code = code * 4u + ((SIGMA == 6 && c == 5u) ? 3u : c - 1u);
    }
    return acgt ? (uint32_t)(code & ((1ull << (2u * a.kmerK)) - 1ull)) : ~0u;
}

// Item i's starting cursor: the k-mer table entry of its error-free first
// part (depth kmerK), else the root. The two lanes of a pair fetch each
// other's 16-B entries cooperatively — each lane 8 B of the even lane's entry,
// then 8 B of the odd lane's, swapped back with DPP — so that a load
// instruction touches at most 32 distinct lines of the 68.7 GB table (address
// translation, not bandwidth, bounds these random lookups: tools/gather_bench).
// Must be called by all lanes of the wave.
template <int SIGMA>
__device__ __forceinline__ uint4 seedOf(const SeedArgs& a, uint32_t i, bool& keep, uint32_t& textPos) {
    keep = i < a.nitems;
    const uint32_t code = seedCode<SIGMA>(a, i);
    const bool need = keep && code != ~0u;
    const bool odd = (threadIdx.x & 1u) != 0u;
    const uint64_t own = (uint64_t)(a.kmer + (need ? code : 0u));
    const uint64_t other = pairSwap64(own);
    const bool otherNeed = pairSwap(need ? 1u : 0u) != 0u;
    const uint64_t addrE = odd ? other : own, addrO = odd ? own : other;
    const bool needE = odd ? otherNeed : need, needO = odd ? need : otherNeed;
    const uint32_t half = odd ? 8u : 0u;
    uint2 rE = make_uint2(0u, 0u), rO = rE;
    if (needE) rE = *reinterpret_cast<const uint2*>(addrE + half);  // even's entry: bytes 0-7 | 8-15
    if (needO) rO = *reinterpret_cast<const uint2*>(addrO + half);  // odd's entry: bytes 0-7 | 8-15
    const uint2 gE = make_uint2(pairSwap(rE.x), pairSwap(rE.y));     // even <- bytes 8-15 of its entry
    const uint2 gO = make_uint2(pairSwap(rO.x), pairSwap(rO.y));     // odd <- bytes 0-7 of its entry
    const uint4 t = odd ? make_uint4(gO.x, gO.y, rO.x, rO.y) : make_uint4(rE.x, rE.y, gE.x, gE.y);
    textPos = t.w;  // SA[lb] when the k-mer occurs once (DeviceIndex::kmerPos)
    if (!need) return make_uint4(0u, 0u, a.n, kDeltaZero);
    keep = t.z != 0u;
    return make_uint4(t.x, t.y, t.z, packMeta(a.kmerK, 0u, OP_MS, OP_MS));
}

// Each block takes 1024 consecutive items per round (4 per thread, so four
// table lookups are in flight per lane) and appends the survivors with one
// atomic per round and output list: seeds for the FM kernel, and text tasks
// for seeds whose k-mer occurs exactly once (toText) — the node the FM kernel
// would hand to the text phase at once.
template <int SIGMA>
__global__ __launch_bounds__(256) void kSeedItems(SeedArgs a) {
    __shared__ uint32_t wcount[2][4], blockBase[2];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t ltMask = (1ull << lane) - 1ull;
    uint64_t cTasks = 0;
    for (uint32_t base = a.itemBegin + blockIdx.x * 1024u; base < a.nitems; base += gridDim.x * 1024u) {  // block-uniform
        uint4 cur[4];
        uint32_t tpos[4];
        bool keep[4], task[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            cur[k] = seedOf<SIGMA>(a, base + k * 256u + threadIdx.x, keep[k], tpos[k]);
            task[k] = keep[k] && a.toText && cur[k].z == 1u && (cur[k].w & 0xFFFFu) < a.m;
            keep[k] = keep[k] && !task[k];
        }
        uint64_t m[4], mt[4];
        uint32_t wsum = 0, wtask = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            m[k] = __ballot(keep[k]);
            mt[k] = __ballot(task[k]);
            wsum += (uint32_t)__popcll(m[k]);
            wtask += (uint32_t)__popcll(mt[k]);
        }
        if (lane == 0) { wcount[0][w] = wsum; wcount[1][w] = wtask; }
        __syncthreads();
        if (threadIdx.x < 2) {
            const uint32_t* wc = wcount[threadIdx.x];
            const uint32_t tot = wc[0] + wc[1] + wc[2] + wc[3];
            blockBase[threadIdx.x] = tot ? atomicAdd(threadIdx.x ? a.taskCount : a.seedCount, tot) : 0u;
        }
        __syncthreads();
        uint32_t slot = blockBase[0], tslot = blockBase[1];
        for (uint32_t j = 0; j < w; ++j) { slot += wcount[0][j]; tslot += wcount[1][j]; }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t item = base + k * 256u + threadIdx.x;
            if (keep[k]) {
                const uint32_t at = slot + (uint32_t)__popcll(m[k] & ltMask);
                a.seeds[at] = cur[k];
                a.seedItem[at] = item;
            }
            if (task[k]) {  // (row, |t| = kmerK, pattern, node meta | search << 24), or with
                            // the text position instead of the row (kTaskPos)
                const uint32_t at = tslot + (uint32_t)__popcll(mt[k] & ltMask);
                const uint32_t pid = item / a.nsearch, sIdx = item - pid * a.nsearch;
                if (at < a.taskCap)
                    a.tasks[at] = make_uint4(a.kmerPos ? tpos[k] : cur[k].x,
                                             (cur[k].w & 0xFFFFu) | (a.kmerPos ? kTaskPos : 0u), pid,
                                             (cur[k].w & 0x00FFFFFFu) | (sIdx << 24));
                else
                    atomicOr(a.flags, 8u);
                ++cTasks;
            }
            slot += (uint32_t)__popcll(m[k]);
            tslot += (uint32_t)__popcll(mt[k]);
        }
        __syncthreads();  // wcount / blockBase reused next round
    }
    if (a.counters && cTasks) {
        atomicAdd(a.counters + 6, (unsigned long long)cTasks);
        if (a.kmerPos) atomicAdd(a.counters + 16, (unsigned long long)cTasks);
    }
}

// =========================================================== phase 1: FM ====

template <int SIGMA, bool EDIT, bool COUNT>
__global__ __launch_bounds__(256) void kSearchFM(SearchArgs a) {
    extern __shared__ uint32_t sch[];
    for (uint32_t i = threadIdx.x; i < a.nsearch * a.m; i += blockDim.x) sch[i] = a.scheme[i];
    __syncthreads();

    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t ltMask = (1ull << lane) - 1ull;
    const bool odd = lane & 1u;
    // DFS stack: the bottom a.ldsDepth levels live in LDS after the scheme
    // table ([level][thread], conflict-free 16-B rows when lanes sit at equal
    // depth), deeper levels spill to HBM ([level][grid thread]).
    uint4* lstk = reinterpret_cast<uint4*>(sch + ((a.nsearch * a.m + 3u) & ~3u));
    const uint32_t ldsDepth = a.ldsDepth;
    uint4* stk = a.stack + gtid;

    // the lane's stack holds entries [bot, sp) in a ring of stackLevels levels
    // (entry d at level d mod stackLevels; bot < stackLevels): pushes and pops
    // at sp, work stealing takes the bottom entry (bot++)
    uint32_t sp = 0, bot = 0, pid = 0, sIdx = 0;
    bool have = false, exhausted = false;
    uint32_t qNext = 0, qEnd = 0, filled = 0;  // wave-uniform
    bool qDone = false;
    SlotRange hitSlots, taskSlots;
    uint4 cur = make_uint4(0, 0, 0, 0);
    uint64_t cNodes = 0, cRank = 0, cLines = 0, cTasks = 0, cIter = 0;
    const uint32_t L = a.stackLevels;
    auto stackGet = [&](uint32_t d) -> uint4 {
        d = d >= L ? d - L : d;
        return d < ldsDepth ? lstk[d * 256u + threadIdx.x] : stk[(size_t)(d - ldsDepth) * T];
    };
    auto stackPut = [&](uint32_t d, const uint4& v) {
        d = d >= L ? d - L : d;
        if (d < ldsDepth) lstk[d * 256u + threadIdx.x] = v;
        else stk[(size_t)(d - ldsDepth) * T] = v;
    };
    // seeds (kSeedItems: starting cursor + item) arrive in chunks of 64, one
    // record per lane, prefetched a chunk ahead so a refill costs no memory trip
    const uint32_t nseeds = *a.seedCount;
    uint4 curRec = make_uint4(0, 0, 0, 0), nextRec = curRec;
    uint32_t curItem = 0, nextItem = 0, nBase = 0, nEnd = 0, qBase = 0;
    bool haveNext = false;
    StripedQueue queue(a.work, nseeds);
    {
        uint32_t b = 0, e = 0;
        if (queue.next(lane, kSeedChunk, b, e)) {
            nBase = b;
            nEnd = e;
            if (b + lane < e) { nextRec = a.seeds[b + lane]; nextItem = a.seedItem[b + lane]; }
            haveNext = true;
        } else {
            qDone = true;
        }
    }

    for (;;) {
        // ---- refill idle lanes from the wave's current seed chunk
        const bool need = !have && sp == bot && !exhausted;
        uint64_t pending = __ballot(need);
        while (pending) {  // wave-uniform
            if (qNext >= qEnd) {
                if (!haveNext) break;
                qBase = nBase;
                qNext = nBase;
                qEnd = nEnd;
                curRec = nextRec;
                curItem = nextItem;
                haveNext = false;
                if (!qDone) {
                    uint32_t b = 0, e = 0;
                    if (!queue.next(lane, kSeedChunk, b, e)) {
                        qDone = true;
                    } else {
                        nBase = b;
                        nEnd = e;
                        if (b + lane < e) { nextRec = a.seeds[b + lane]; nextItem = a.seedItem[b + lane]; }
                        haveNext = true;
                    }
                }
                if (qNext >= qEnd) continue;
            }
            const uint32_t take = min(qEnd - qNext, (uint32_t)__popcll(pending));
            const uint32_t rank = (uint32_t)__popcll(pending & ltMask);
            const bool mine = ((pending >> lane) & 1ull) && rank < take;
            const uint32_t src = (qNext - qBase + rank) & 63u;
            const uint4 sd = make_uint4(__shfl(curRec.x, src), __shfl(curRec.y, src), __shfl(curRec.z, src),
                                        __shfl(curRec.w, src));
            const uint32_t item = __shfl(curItem, src);
            if (mine) {
                pid = item / a.nsearch;
                sIdx = item - pid * a.nsearch;
                cur = sd;
                have = true;
            }
            pending &= ~__ballot(mine);
            qNext += take;
        }
        if (qDone && !haveNext && qNext >= qEnd && need && !have) exhausted = true;
        if (!have && sp > bot) {
            --sp;
            cur = stackGet(sp);
            have = true;
        }
        if (sp == bot) sp = bot = 0;
        // ---- work stealing inside the wave once the seed queue is dry (wave-
        // uniform: the queue state is the wave's). The DFS of one seed varies
        // by orders of magnitude in size (repeats, and from the root every
        // search ranks thousands of nodes at k = 3), so a launch otherwise ends
        // with most lanes idle beside a few long ones (reference execution at
        // C5: lanes busy 0.49). An idle lane takes the bottom (shallowest, so
        // largest) stack entry of the r-th busy lane, with its pattern id and
        // search by shuffle; the entry's subtree is the same DFS whichever lane
        // runs it, so the leaves are too.
        if (a.stealAt && qDone && !haveNext && qNext >= qEnd) {
            const bool thief = !have;
            const uint64_t I = __ballot(thief);
            const uint64_t D = __ballot(have && sp > bot);
            const uint32_t nI = (uint32_t)__popcll(I), nD = (uint32_t)__popcll(D);
            if (nI >= a.stealAt && nD) {  // wave-uniform
                const uint32_t n = min(nI, nD);
                const uint32_t r = (uint32_t)__popcll(I & ltMask);
                uint32_t donor = 0, rr = r;
                uint64_t dm = D;
#pragma unroll
                for (uint32_t w = 32; w; w >>= 1) {  // the r-th set bit of D
                    const uint32_t c = (uint32_t)__popcll(dm & ((1ull << w) - 1ull));
                    if (rr >= c) { rr -= c; dm >>= w; donor += w; }
                }
                const bool takes = thief && r < n;
                donor = takes ? donor : lane;
                const uint32_t dPid = __shfl(pid, donor), dS = __shfl(sIdx, donor), dBot = __shfl(bot, donor);
                if (takes) {
                    const uint32_t dt = (threadIdx.x & ~63u) | donor;
                    const uint32_t lv = dBot;  // < L
                    if (lv < ldsDepth) cur = lstk[lv * 256u + dt];
                    else cur = loadGlobal4(a.stack + (size_t)(lv - ldsDepth) * T + (gtid & ~63u) + donor);
                    pid = dPid;
                    sIdx = dS;
                    have = true;
                }
                // the thieves' reads complete before a donor's later pushes
                // can reuse the level (its stack emptied and reset)
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (((D >> lane) & 1ull) && (uint32_t)__popcll(D & ltMask) < n && ++bot == L) {
                    bot = 0;
                    sp -= L;
                }
            }
        }
        if (!__any(have)) break;
        if (COUNT && lane == 0) ++cIter;

        const uint32_t pos = cur.w & 0xFFFFu;
        // ---- leaves -> hit buffer
        {
            const bool leaf = have && pos == a.m;
            uint32_t slot;
            if (hitSlots.take(leaf, lane, ltMask, a.hitCount, slot) && leaf) {
                if (slot < a.hitCap) {
                    a.hits[slot] = make_uint4(pid, cur.x, cur.z, (cur.w >> 16) & 0xFu);
                    a.rank[slot] = atomicAdd(a.qcnt + pid, cur.z);  // its first row's place in the query's segment
                } else {
                    atomicOr(a.flags, 2u);
                }
                have = false;
                ++filled;
            }
        }
        // ---- small intervals -> one text task per row (phase 2)
        if (a.split) {
            const bool conv = have && cur.z <= a.split;
            const uint32_t tlen = pos + metaDelta(cur.w) - 16u;  // |t|
            for (uint32_t j = 0; __any(conv && j < cur.z); ++j) {  // wave-uniform trip count
                const bool want = conv && j < cur.z;
                uint32_t slot;
                if (taskSlots.take(want, lane, ltMask, a.taskCount, slot) && want) {
                    if (slot < a.taskCap)
                        a.tasks[slot] = make_uint4(cur.x + j, tlen, pid, (cur.w & 0x00FFFFFFu) | (sIdx << 24));
                    else atomicOr(a.flags, 8u);
                    if (COUNT) ++cTasks;
                }
            }
            if (conv) have = false;
        }

        // ---- decode the node (per lane)
        uint32_t e = 0, lastL = 0, lastR = 0, cq = 0;
        bool right = false, matchOK = false, misOK = false, delOK = false, insOK = false;
        uint32_t lo = 0, hi = 0;
        bool needA = false, needB = false;
        if (have) {
            e = (cur.w >> 16) & 0xFu;
            lastL = (cur.w >> 20) & 3u;
            lastR = (cur.w >> 22) & 3u;
            const uint32_t se = sch[sIdx * a.m + pos];
            const uint32_t q = se & 0xFFFFu, lb = (se >> 16) & 0xFu, ub = (se >> 20) & 0xFu;
            right = (se >> 24) & 1u;
            cq = nib(a.pats[(size_t)pid * a.patWords + (q >> 3)], q);
            const uint32_t side = right ? lastR : lastL;
            matchOK = lb <= e && e <= ub;
            misOK = lb <= e + 1 && e + 1 <= ub;
            delOK = EDIT && pos > 0 && e + 1 <= ub && side != OP_I;
            insOK = EDIT && misOK && side != OP_D;
            lo = right ? cur.y : cur.x;
            hi = lo + cur.z;
            needA = matchOK || misOK || delOK;
            needB = needA && (hi >> 6) != (lo >> 6);
        }

        // ---- pair-cooperative Occ line fetch (wave-uniform)
        const uint64_t ownA = (uint64_t)(right ? a.occR : a.occF) + (uint64_t)(lo >> 6) * 64u;
        const uint64_t ownB = (uint64_t)(right ? a.occR : a.occF) + (uint64_t)(hi >> 6) * 64u;
        uint32_t ca[5], cb[5];
        uint64_t pa[3], pb[3];
        fetchLinePair(ownA, needA, odd, ca, pa);
        fetchLinePair(ownB, needB, odd, cb, pb);

        if (have) {
            if (COUNT) ++cNodes;
            // child c = (fx[c], fy[c], occ[c]): forward / reverse lower bounds
            uint32_t occ[SIGMA], fx[SIGMA], fy[SIGMA];
#pragma unroll
            for (int c = 0; c < SIGMA; ++c) occ[c] = fx[c] = fy[c] = 0;
            if (needA) {
                if (!needB) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) cb[i] = ca[i];
                    pb[0] = pa[0]; pb[1] = pa[1]; pb[2] = pa[2];
                }
                if (COUNT) { ++cRank; cLines += needB ? 2 : 1; }
                const uint64_t ml = lowMask(lo & 63u), mh = lowMask(hi & 63u);
                uint32_t sum = 0, base[SIGMA];
#pragma unroll
                for (int c = 1; c < SIGMA; ++c) {
                    const uint32_t rl = ca[c - 1] + (uint32_t)__popcll(symMask(pa, c) & ml);
                    const uint32_t rh = cb[c - 1] + (uint32_t)__popcll(symMask(pb, c) & mh);
                    occ[c] = rh - rl;
                    base[c] = a.C[c] + rl;
                    sum += occ[c];
                }
                // bidirectional update: the other side moves by the occurrences
                // of the smaller symbols, '$' first
                uint32_t acc = (right ? cur.x : cur.y) + (cur.z - sum);
#pragma unroll
                for (int c = 1; c < SIGMA; ++c) {
                    fx[c] = right ? acc : base[c];
                    fy[c] = right ? base[c] : acc;
                    acc += occ[c];
                }
            }
            const uint32_t dl = metaDelta(cur.w);
            auto mk = [&](int c, uint32_t kind) -> uint4 {
                uint32_t f = 0, g = 0, o = 0;
#pragma unroll
                for (int s = 1; s < SIGMA; ++s)
                    if (s == c) { f = fx[s]; g = fy[s]; o = occ[s]; }
                return make_uint4(f, g, o, childMeta(pos, e, lastL, lastR, right, dl, kind));
            };
            auto push = [&](const uint4& v) {
                if (sp - bot < a.stackCap) {
                    stackPut(sp, v);
                    ++sp;
                } else {
                    atomicOr(a.flags, 1u);
                }
            };
            const uint4 ins = make_uint4(cur.x, cur.y, cur.z, childMeta(pos, e, lastL, lastR, right, dl, 3));
            uint4 next = make_uint4(0, 0, 0, 0);
            have = expandChildren<SIGMA>(occ, cq, matchOK, misOK, delOK, insOK, ins, mk, push, next);
            cur = next;
        }
    }
    hitSlots.close(lane, a.hits, a.hitCap);
    taskSlots.close(lane, a.tasks, a.taskCap);
    if (filled) atomicAdd(a.filled, filled);  // per-lane counts
    if (COUNT) {
        atomicAdd(a.counters + 0, (unsigned long long)cNodes);
        atomicAdd(a.counters + 1, (unsigned long long)cRank);
        atomicAdd(a.counters + 2, (unsigned long long)cLines);
        atomicAdd(a.counters + 6, (unsigned long long)cTasks);
        if (cIter) atomicAdd(a.counters + 7, (unsigned long long)cIter);
    }
}

// ========================================================= phase 2: text ====
//
// LDS: table[S*m] (uint2: packed scheme | run << 25, covered [a, b)) | per
// lane, interleaved so that the lanes of a wave hit consecutive banks at
// equal offsets:
//   window  (winBlocks blocks of 32 symbols)     W[(3j+b)*256 + t], plane b
//   pattern (patBlocks blocks of 32 symbols)     P[(3j+b)*256 + t]
//   stack   (stackCap entries)                   S[d*256 + t]: uint2, or one
//           packed word (PK: m <= 127, window <= 256 symbols, e <= 7)
//
// A lane's state is one DFS node `cur` (x = window offsets xo | yo << 16 of
// the text t matched so far, y = pos | e << 16 | lastL << 20 | lastR << 22).
// Every micro-step is straight-line code — one stack read, one table read,
// 8-symbol reads of the window on both sides of the span and of the pattern at
// pi[pos] and pi[pos+1], three stack writes — so the
// lanes of a wave stay converged. A node with e == u[pos] has no error child
// in the forced run of positions that follows it (table `run`), so it takes
// up to 8 forced matches at once: the DFS visits the same chain of nodes,
// one micro-step per 16 of them.



// ---- runs of symbols as bit masks: bit j = chain symbol j. Symbols come as
// 3 bit planes (device_index.h), so the per-symbol equality of 32 symbols is
// three word xors; the chain logic uses the low 16 bits.
constexpr uint32_t kRun = 32;              // symbols per micro-step run (a forced node's match budget)
constexpr uint32_t kRunMask = 0xFFFFFFFFu;
// chain positions per micro-step of a node whose error children are forced:
// the forced-run check of an error child at chain node i reads symbols
// i .. i + 7 of the 32 (kChain + 7 <= kRun)
constexpr uint32_t kChain = 25;
__device__ __forceinline__ uint32_t onesR(uint32_t n) {  // symbols [0, n), capped at kRun
    return n >= kRun ? kRunMask : (1u << n) - 1u;
}
__device__ __forceinline__ uint32_t beyondR(uint32_t n) { return kRunMask & ~onesR(n); }  // symbols >= n
// bit j set iff bits j .. j+6 are all set (7 consecutive matches from j)
__device__ __forceinline__ uint32_t run7(uint32_t m) {
    const uint32_t m2 = m & (m >> 1), m4 = m2 & (m2 >> 2);
    return m4 & (m2 >> 4) & (m >> 6);
}
struct Planes { uint32_t b0, b1, b2; };
__device__ __forceinline__ uint32_t eqm(const Planes& p, const Planes& t) {
    return ~((p.b0 ^ t.b0) | (p.b1 ^ t.b1) | (p.b2 ^ t.b2));
}
__device__ __forceinline__ Planes shr1(const Planes& p) { return {p.b0 >> 1, p.b1 >> 1, p.b2 >> 1}; }
__device__ __forceinline__ Planes shr2(const Planes& p) { return {p.b0 >> 2, p.b1 >> 2, p.b2 >> 2}; }
// 32 symbols from offset o of a lane's interleaved plane array (block i, plane
// b at word (3i + b) * 256). o may be negative (down to -32): reads may run
// past either end of the array into the lane's neighbouring LDS regions; callers
// mask.
__device__ __forceinline__ uint32_t read32(const uint32_t* A, int o, uint32_t b) {
    const int i = o >> 5;
    return __builtin_amdgcn_alignbit(A[(3 * i + 3 + (int)b) * 256], A[(3 * i + (int)b) * 256], (uint32_t)o & 31u);
}
// 32 symbols in chain order: right (fwd) from o, or left ending at o - 1 and
// reversed (back: bit j = symbol o - 1 - j). Symbols outside the array are
// whatever the LDS holds there (the window's block -1 is the table region,
// kTextTableMin words, the pattern's is the window): the window's are masked
// by its `avail`, the pattern's lie beyond the pattern, which the chain logic
// never uses (tests/text_model.py reads arbitrary symbols there).
__device__ __forceinline__ Planes chain32(const uint32_t* A, uint32_t o, bool fwd) {
    const int off = (int)o - (fwd ? 0 : 32);
    Planes r;
    uint32_t v[3];
#pragma unroll
    for (uint32_t b = 0; b < 3; ++b) {
        const uint32_t w = read32(A, off, b);
        v[b] = fwd ? w : __builtin_bitreverse32(w);
    }
    r.b0 = v[0]; r.b1 = v[1]; r.b2 = v[2];
    return r;
}

// Raw buffer resource over [base, base + bytes) (gfx9 dword3): loads at an
// offset past the end return 0 without a memory request, so guarded loads
// need no branch (and no wait at a branch join).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bufferOf(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
constexpr uint32_t kBufOOB = 0xFFFFFFFFu;  // offset of a load that returns 0

// Copy two block arrays (window, pattern) from global memory into this lane's
// interleaved LDS slots (3 words per block): all loads of up to 8 blocks of
// each array are issued before the first store, so a task start costs one
// memory round trip for m <~ 190.
__device__ __forceinline__ void copyBlocks(uint32_t* DA, __amdgpu_buffer_rsrc_t RA, uint32_t offA, uint32_t na,
                                           uint32_t* DB, __amdgpu_buffer_rsrc_t RB, uint32_t offB, uint32_t nb) {
    const uint32_t n = max(na, nb);
    for (uint32_t c = 0; c < n; c += 8) {
        decltype(__builtin_amdgcn_raw_buffer_load_b128(RA, 0u, 0, 0)) va[8], vb[8];
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t j = c + i;
            va[i] = __builtin_amdgcn_raw_buffer_load_b128(RA, j < na ? offA + 16u * j : kBufOOB, 0, 0);
            vb[i] = __builtin_amdgcn_raw_buffer_load_b128(RB, j < nb ? offB + 16u * j : kBufOOB, 0, 0);
        }
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t j = c + i;
            if (j < na) { uint32_t* D = DA + 3u * j * 256u; D[0] = va[i][0]; D[256] = va[i][1]; D[512] = va[i][2]; }
            if (j < nb) { uint32_t* D = DB + 3u * j * 256u; D[0] = vb[i][0]; D[256] = vb[i][1]; D[512] = vb[i][2]; }
        }
    }
}

// Same, but the window starts at any symbol: na blocks come from na + 1
// source blocks funnel-shifted by sh symbols (na + 1 <= 8, nb <= 8).
__device__ __forceinline__ void copyBlocksShifted(uint32_t* DA, __amdgpu_buffer_rsrc_t RA, uint32_t offA, uint32_t sh,
                                                  uint32_t na, uint32_t* DB, __amdgpu_buffer_rsrc_t RB, uint32_t offB,
                                                  uint32_t nb) {
    decltype(__builtin_amdgcn_raw_buffer_load_b128(RA, 0u, 0, 0)) va[8], vb[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        va[j] = __builtin_amdgcn_raw_buffer_load_b128(RA, j <= na ? offA + 16u * j : kBufOOB, 0, 0);
        vb[j] = __builtin_amdgcn_raw_buffer_load_b128(RB, j < nb ? offB + 16u * j : kBufOOB, 0, 0);
    }
#pragma unroll
    for (uint32_t j = 0; j < 7; ++j)
        if (j < na) {
            uint32_t* D = DA + 3u * j * 256u;
            D[0] = __builtin_amdgcn_alignbit(va[j + 1][0], va[j][0], sh);
            D[256] = __builtin_amdgcn_alignbit(va[j + 1][1], va[j][1], sh);
            D[512] = __builtin_amdgcn_alignbit(va[j + 1][2], va[j][2], sh);
        }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
        if (j < nb) { uint32_t* D = DB + 3u * j * 256u; D[0] = vb[j][0]; D[256] = vb[j][1]; D[512] = vb[j][2]; }
}

// SHAPE fixes the window and pattern block counts at compile time, so that
// the task-start copy is straight-line code with no per-block conditions (the
// generic form, SHAPE 0, keeps ~30 block masks in spilled SGPRs and reloads
// them at every task start: 1882 against 1311 instructions, 101 against 85
// VGPRs; C3 850-863M -> 886-893M reads/s).
//   1: window 4 blocks at an exact start, pattern 4 blocks (C2, C3: m = 100)
//   2: window 9 blocks block-aligned, pattern 8 blocks (C5: m = 250, k = 3)
struct TextShape { uint32_t win, pat; bool exact; };
__host__ __device__ constexpr TextShape textShape(int shape) {
    return shape == 1 ? TextShape{4, 4, true} : shape == 2 ? TextShape{9, 8, false} : TextShape{0, 0, false};
}


// ---- kSearchTextBatch: the text phase of one batch per launch. Its tasks
// [*taskBegin, *taskCount) of the slot's list come from a striped queue; a
// lane takes a task (text position, or SA row read here), copies the window
// and pattern to LDS and runs the subtree's DFS against the text; leaves are
// hits (qid, text position, e | kPosKnown), each ranked in its query's
// segment as it is written (kLocate places them). (Round 5's persistent
// variant, one launch per pass, measured 2-3x slower and was removed in r6:
// DESIGN.md §3.4.)
template <int SIGMA, bool EDIT, bool COUNT, int SHAPE = 0>
__global__ __launch_bounds__(256) void kSearchTextBatch(TextBatchArgs a) {
    extern __shared__ uint32_t lds[];
    uint2* SC = reinterpret_cast<uint2*>(lds);
    uint32_t* slot = lds + a.tableWords;  // >= kTextTableMin: the window's block -1 stays in LDS
    for (uint32_t i = threadIdx.x; i < a.nsearch * a.m; i += blockDim.x) SC[i] = a.table[i];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t ltMask = (1ull << lane) - 1ull;
    constexpr TextShape kShape = textShape(SHAPE);
    const uint32_t winBlocks = SHAPE ? kShape.win : a.winBlocks, patBlocks = SHAPE ? kShape.pat : a.patBlocks;
    const bool exactWindow = SHAPE ? kShape.exact : a.exactWindow != 0u;
    uint32_t* W = slot + threadIdx.x;
    uint32_t* P = slot + 3u * winBlocks * 256u + threadIdx.x;
    uint2* S = reinterpret_cast<uint2*>(slot + 3u * (winBlocks + patBlocks) * 256u) + threadIdx.x;
    auto stackGet = [&](uint32_t d) -> uint2 { return S[d * 256u]; };
    auto stackPut = [&](uint32_t d, const uint2& v) { S[d * 256u] = v; };
    const uint32_t winLen = winBlocks * 32u;
    const __amdgpu_buffer_rsrc_t textBuf = bufferOf(a.text3, a.text3Bytes);
    const __amdgpu_buffer_rsrc_t patBuf = bufferOf(a.pats3, a.pats3Bytes);
    const uint32_t m = a.m;
    // this launch's tasks: [tBase, taskCount) of the batch's list
    const uint32_t tEnd = min(*a.taskCount, a.taskCap);
    const uint32_t tBase = a.taskBegin ? min(*a.taskBegin, tEnd) : 0u;
    const uint32_t ntasks = tEnd - tBase;
    const uint4* tasks = a.tasks + tBase;

    uint32_t sp = 0, pid = 0, wb = 0, sBase = 0;
    bool have = false, exhausted = false, bad = false;
    uint32_t qNext = 0, qEnd = 0, filled = 0;
    bool qDone = false;
    // task chunks: the current one's records (one per lane) and the next one's,
    // prefetched a chunk ahead so a refill needs no dependent task read
    uint4 curRec = make_uint4(0, 0, 0, 0), nextRec = curRec;
    uint32_t nBase = 0, nEnd = 0, qBase = 0;
    bool haveNext = false;
    // The prefetched chunk's records still hold SA rows. Their text positions
    // are read at the next refill, beside its window loads (one round trip for
    // both), or at the latest when the chunk becomes current.
    bool nextRaw = false;
    auto resolveNext = [&]() {
        if (nextRaw) {  // wave-uniform
            if (nBase + lane < nEnd && !(nextRec.y & kTaskPos)) nextRec.x = a.sa[nextRec.x];
            nextRaw = false;
        }
    };
    StripedQueue queue(a.work, ntasks);
    {
        uint32_t b = 0, e = 0;
        if (queue.next(lane, kTaskChunk, b, e)) {
            nBase = b;
            nEnd = e;
            if (b + lane < e) nextRec = tasks[b + lane];
            haveNext = true;
            nextRaw = true;
        } else {
            qDone = true;
        }
    }
    SlotRange hitSlots;
    uint32_t rankSlot = ~0u, rankVal = 0;  // the lane's last hit whose rank is not stored yet
    uint2 cur = make_uint2(0, 0);
    uint64_t cNodes = 0, tIter = 0, tActive = 0, tRefill = 0, cCmp = 0, cSteps = 0;
    uint64_t cyRefill = 0, cyStep = 0, cyEmit = 0, t0 = 0, cSteal = 0;
    // (count mode, a.probe) the first launch's wave lives on the wall clock:
    // the queue seen drained, iterations and busy lanes before / after it.
    // Only in count mode: it costs the product kernel 14 VGPRs and 12 SGPR spills.
    constexpr bool kProbe = COUNT;
    __shared__ uint64_t wBorn[4], wDrain[4];
    if (kProbe && a.probe && lane == 0) wBorn[threadIdx.x >> 6] = wall_clock64(), wDrain[threadIdx.x >> 6] = 0;
    uint32_t pIterPre = 0, pIterPost = 0, pActPre = 0, pActPost = 0;
    uint64_t pwPreA = 0, pwPreB = 0, pwPostA = 0, pwPostB = 0, pw0 = 0, pw1 = 0;

    for (;;) {
        if (kProbe && a.probe) pw0 = wall_clock64();
        // Starting a task costs a global round trip (window + pattern) that
        // stalls the whole wave, so idle lanes are refilled in batches: once
        // refillAt lanes are idle (or nothing else is left).
        if (COUNT) t0 = clock64();
        const bool idle = !have && sp == 0 && !exhausted;
        const uint64_t idleMask = __ballot(idle);
        const bool busy = __any(have || sp > 0);
        const bool refill = !busy || __popcll(idleMask) >= a.refillAt;
        const bool need = refill && idle;
        uint64_t pending = refill ? idleMask : 0ull;
        if (pending) resolveNext();
        while (pending) {  // wave-uniform
            if (qNext >= qEnd) {
                // switch to the prefetched chunk, prefetch the one after it
                if (!haveNext) break;
                resolveNext();
                qBase = nBase;
                qNext = nBase;
                qEnd = nEnd;
                curRec = nextRec;
                haveNext = false;
                if (!qDone) {
                    uint32_t b = 0, e = 0;
                    if (!queue.next(lane, kTaskChunk, b, e)) {
                        qDone = true;
                    } else {
                        nBase = b;
                        nEnd = e;
                        if (b + lane < e) nextRec = tasks[b + lane];
                        haveNext = true;
                        nextRaw = true;
                    }
                }
                if (qNext >= qEnd) continue;
            }
            const uint32_t take = min(qEnd - qNext, (uint32_t)__popcll(pending));
            const uint32_t rank = (uint32_t)__popcll(pending & ltMask);
            const bool mine = ((pending >> lane) & 1ull) && rank < take;
            // the chunk's task records sit one per lane: fetch ours by shuffle
            const uint32_t srcLane = (qNext - qBase + rank) & 63u;
            const uint4 t = make_uint4(__shfl(curRec.x, srcLane), __shfl(curRec.y, srcLane),
                                       __shfl(curRec.z, srcLane), __shfl(curRec.w, srcLane));
            if (mine && t.y != 0u) {  // |t| = 0: an unused reserved slot (SlotRange::close)
                // ---- start a task (x = its text position): copy the pattern
                // and the text window its subtree can reach
                const uint32_t x = t.x;
                pid = t.z;
                sBase = (t.w >> 24) * m;
                const uint32_t meta = t.w & 0x00FFFFFFu;
                const uint32_t pos = meta & 0xFFFFu, e = (meta >> 16) & 0xFu;
                const uint32_t ca = SC[sBase + pos].y & 0xFFFu;
                const uint32_t K = (SC[sBase + m - 1u].x >> 20) & 0xFu;
                const uint32_t left = ca + (K > e ? K - e : 0u);  // text the left side can still consume
                wb = x > left ? x - left : 0u;  // window start
                if (exactWindow) {              // at wb: m + 2k symbols fit in winBlocks blocks
                    copyBlocksShifted(W, textBuf, (wb >> 5) * 16u, wb & 31u, winBlocks, P, patBuf,
                                      pid * patBlocks * 16u, patBlocks);
                } else {                        // at the block start below wb (31 more symbols)
                    wb &= ~31u;
                    copyBlocks(W, textBuf, (wb >> 5) * 16u, winBlocks, P, patBuf, pid * patBlocks * 16u, patBlocks);
                }
                cur = make_uint2((x - wb) | ((x + (t.y & 0xFFFFu) - wb) << 16), meta);
                have = true;
            }
            pending &= ~__ballot(mine);
            qNext += take;
        }
        if (qDone && !haveNext && qNext >= qEnd && need && !have) exhausted = true;
        // ---- work stealing inside the wave once the task queue is dry (wave-
        // uniform: the queue state is the wave's). A launch ends on its longest
        // subtrees, each on one lane while the others idle (C5: lanes busy
        // 0.655 of the time); an idle lane takes the bottom (shallowest, so
        // largest) stack entry of a busy lane, with that lane's window and
        // pattern copied slot to slot in LDS, and the task state (pattern id,
        // window start, scheme row) by shuffle. The DFS of the entry is the
        // same whichever lane runs it, so the hits are too.
        if (a.stealAt && qDone && !haveNext && qNext >= qEnd) {
            const bool thief = !have && sp == 0u;
            const uint64_t I = __ballot(thief);
            const uint64_t D = __ballot(sp >= 2u || (sp == 1u && have));
            const uint32_t nI = (uint32_t)__popcll(I), nD = (uint32_t)__popcll(D);
            if (nI >= a.stealAt && nD) {  // wave-uniform
                const uint32_t n = min(nI, nD);
                const uint32_t r = (uint32_t)__popcll(I & ltMask);
                // donor of thief rank r: the r-th set bit of D
                uint32_t donor = 0, rr = r;
                uint64_t dm = D;
#pragma unroll
                for (uint32_t w = 32; w; w >>= 1) {
                    const uint32_t c = (uint32_t)__popcll(dm & ((1ull << w) - 1ull));
                    if (rr >= c) { rr -= c; dm >>= w; donor += w; }
                }
                const bool takes = thief && r < n;
                donor = takes ? donor : lane;
                const uint32_t dPid = __shfl(pid, donor), dWb = __shfl(wb, donor), dBase = __shfl(sBase, donor);
                const uint32_t dTid = (threadIdx.x & ~63u) | donor;
                if (takes) {
                    const uint32_t* src = slot + dTid;
                    uint32_t* dst = slot + threadIdx.x;
                    for (uint32_t k = 0; k < 3u * (winBlocks + patBlocks); ++k) dst[k * 256u] = src[k * 256u];
                    const uint2 node = reinterpret_cast<const uint2*>(slot + 3u * (winBlocks + patBlocks) * 256u)[dTid];
                    cur = node;
                    pid = dPid;
                    wb = dWb;
                    sBase = dBase;
                    have = true;
                    if (COUNT) ++cSteal;
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                // donors (rank < n) drop their bottom entry
                const bool gives = ((D >> lane) & 1ull) && (uint32_t)__popcll(D & ltMask) < n;
                if (gives) {
                    for (uint32_t d = 1; d < sp; ++d) stackPut(d - 1u, stackGet(d));
                    --sp;
                }
            }
        }
        if (!__any(have || sp > 0 || (!exhausted && (!qDone || haveNext || qNext < qEnd)))) break;  // nothing left
        if (kProbe && a.probe) {
            if (qDone && lane == 0 && wDrain[threadIdx.x >> 6] == 0) wDrain[threadIdx.x >> 6] = wall_clock64();
            const uint32_t act = (uint32_t)__popcll(__ballot(have || sp > 0));
            if (qDone) { ++pIterPost; pActPost += act; } else { ++pIterPre; pActPre += act; }
            pw1 = wall_clock64();
        }
        if (COUNT) {
            const uint64_t act = __ballot(have || sp > 0);
            if (lane == 0) { ++tIter; tActive += (uint64_t)__popcll(act); tRefill += refill ? 1u : 0u; }
            const uint64_t t1 = clock64();
            cyRefill += t1 - t0;
            t0 = t1;
        }

        // ---- up to a.steps micro-steps per lane; a lane that reaches a leaf
        // holds it (stalls) until the emission below
        bool leaf = false;
        uint32_t leafStart = 0, leafE = 0;
        for (uint32_t step = 0; step < a.steps; ++step) {
            const bool pop = !have && !leaf && sp > 0;
            const uint2 top = stackGet(pop ? sp - 1u : 0u);
            if (pop) { cur = top; --sp; have = true; }
            const bool live = have && !leaf;
            if (!__any(live)) break;  // wave-uniform

            const uint32_t pos = cur.y & 0xFFFFu;
            const uint32_t xo = cur.x & 0xFFFFu, yo = cur.x >> 16;
            const uint32_t e = (cur.y >> 16) & 0xFu;
            const uint32_t lastL = (cur.y >> 20) & 3u, lastR = (cur.y >> 22) & 3u;
            const uint2 tab = SC[sBase + min(pos, m - 1u)];
            const uint32_t t0 = tab.x;
            const uint32_t q0 = t0 & 0xFFFFu, lb0 = (t0 >> 16) & 0xFu, ub0 = (t0 >> 20) & 0xFu;
            const bool r0 = (t0 >> 24) & 1u;
            const uint32_t run0 = t0 >> 25, same0 = (tab.y >> 24) & 0x7Fu;

            // ---- pattern symbols from pi[pos] in this step's direction and
            // the text symbols beyond the span on that side, both in chain
            // order (symbol j of the chain in bit j); text past the window
            // edge or before the text start reads as 0 and never matches.
            // One read each at a side-dependent offset (a left run ends at the
            // position and is bit-reversed), so the lanes of both sides share it
            const Planes P16 = chain32(P, r0 ? q0 : q0 + 1u, r0);
            const Planes T16 = chain32(W, r0 ? yo : xo, r0);
            const uint32_t avail = r0 ? (winLen > yo ? winLen - yo : 0u) : xo;
            const uint32_t VT = onesR(avail);
            const uint32_t E0 = eqm(P16, T16) & VT;                 // p_j == t_j     (M chain, S runs)
            const uint32_t ED = eqm(P16, shr1(T16)) & (VT >> 1);    // p_j == t_{j+1} (D runs)
            const uint32_t EI = eqm(shr1(P16), T16) & VT;           // p_{j+1} == t_j (I runs)
            const uint32_t TZ = (T16.b0 | T16.b1 | T16.b2) & VT;    // t_j is a symbol (not '$' / edge)

            const bool atLeaf = live && pos == m;
            const bool node = live && pos < m;
            const bool forced = e == ub0;          // no error child here or in the rest of the run
            const bool kidsF = e + 1u == ub0;      // the error children are forced nodes
            const bool mOK = lb0 <= e && e <= ub0;
            const bool misOK = lb0 <= e + 1u && e + 1u <= ub0;
            const uint32_t side = r0 ? lastR : lastL;
            // chain budget: a forced node matches up to kRun symbols; a node
            // whose error children are forced walks up to kChain positions of
            // its match chain (same direction, l and u), checking every error
            // child's forced run on the way; any other node is expanded alone
            const uint32_t B = forced ? min(run0, kRun)
                                      : (kidsF ? max(1u, min(min(same0, run0 - 1u), kChain)) : 1u);
            const uint32_t miss = ~E0 & kRunMask;
            const uint32_t L = mOK ? min(B, miss ? (uint32_t)__builtin_ctz(miss) : kRun) : 0u;

            // ---- error children of the chain nodes i < NN (node L = the mismatch)
            const uint32_t NN = L < B ? L + 1u : B;
            const uint32_t nodesM = node && !forced ? onesR(NN) : 0u;  // leaves / idle lanes: none
            const uint32_t first = 1u;  // chain node 0 (= this node)
            uint32_t Dm = EDIT ? (nodesM & TZ) : 0u;
            if (pos == 0u || side == OP_I) Dm &= ~first;
            uint32_t Im = EDIT && misOK ? nodesM : 0u;
            if (side == OP_D) Im &= ~first;
            // S at the first mismatch (not where M is merely disallowed: l > e)
            bool Sx = node && !forced && L < B && misOK && ((TZ & ~E0) >> L) & 1u;
            // forced runs: a child at e + 1 = u is forced for the rest of the run,
            // and survives only if min(7, rest of the run) symbols match on its
            // diagonal (positions past the run count as matches): R7x bit j =
            // that check for a run starting at chain position j on diagonal x
            const uint32_t bR = beyondR(run0), bR1 = beyondR(run0 - 1u);
            const uint32_t R7E0 = run7(E0 | bR), R7ED = run7(ED | bR), R7EI = run7(EI | bR1);
            if (kidsF) {
                // D at i: p[i..] vs t[i+1..]; I at i: p[i+1..] vs t[i..]; S at L: p[L+1..] vs t[L+1..]
                Dm &= R7ED;
                Im &= R7EI;
                Sx = Sx && ((R7E0 >> (L + 1u)) & 1u);
            }
            if (EDIT && node && e + 2u == ub0) {
                // A node expanded alone whose error children are chain nodes:
                // keep only the children whose subtree outlives their own first
                // step. A child does if its match chain leaves the run or the
                // 32 symbols read (chain length > kRun - 9), or one of its own
                // error children (forced) passes the check above on its
                // diagonal; no I right after D, no D right after I (policy P0).
                // tests/text_model.py holds this to the plain DFS.
                const uint32_t ED2 = eqm(P16, shr2(T16)) & (VT >> 2);   // p_j == t_{j+2}
                const uint32_t EI2 = eqm(shr2(P16), T16) & VT;          // p_{j+2} == t_j
                const uint32_t bR2 = run0 >= 2u ? beyondR(run0 - 2u) : kRunMask;
                const uint32_t R7ED2 = run7(ED2 | bR), R7EI2 = run7(EI2 | bR2);
                const uint32_t I2after = (R7E0 >> 1) & ~1u;  // bit j: I2 (back to diagonal 0) at chain node j > 0
                constexpr uint32_t kLim = kRun - 9u;
                if (Dm & first) {  // D child: p_j vs t_{j+1}
                    const uint32_t LD = (uint32_t)__builtin_ctz(~ED);
                    const bool keep = LD >= run0 || LD > kLim || ((R7ED >> (LD + 1u)) & 1u) ||
                                      ((R7ED2 | I2after) & onesR(LD + 1u)) != 0u;
                    if (!keep) Dm &= ~first;
                }
                if (Im & first) {  // I child: p_{x+1} vs t_x
                    const uint32_t LI = ~EI ? (uint32_t)__builtin_ctz(~EI) : kRun;
                    const bool keep = LI + 1u >= run0 || LI > kLim || ((R7EI >> (LI + 1u)) & 1u) ||
                                      ((I2after | R7EI2) & onesR(LI + 1u)) != 0u;
                    if (!keep) Im &= ~first;
                }
                if (Sx) {  // S child at the mismatch L = 0: p_x vs t_x, x >= 1
                    const uint32_t rest = ~E0 & ~1u;
                    const uint32_t LS = rest ? (uint32_t)__builtin_ctz(rest) : kRun;
                    Sx = LS >= run0 || LS > kLim || ((R7E0 >> (LS + 1u)) & 1u) ||
                         ((R7ED | R7EI) & ~1u & onesR(LS + 1u)) != 0u;
                }
            }
            const bool contM = node && L >= B;  // the match chain continues at pos + B
            uint32_t nSurv = (uint32_t)__popc(Dm) + (uint32_t)__popc(Im) + (Sx ? 1u : 0u);
            // the lane continues with one child and stacks the others: a
            // surviving error child first, the match chain below it
            uint32_t Bc = B;
            // Stack invariant (stackCap = 2k + 2): a node that stacks entries
            // with e errors finds sp <= 2e + 2. One node expanded alone stacks
            // <= 2; a chain may stack more only while the child it continues
            // with (e + 1) still finds sp <= 2(e + 1) + 2.
            if (nSurv && sp + nSurv + (contM ? 1u : 0u) - 1u > 2u * e + 4u) {
                // not enough stack for this chain: expand its first node only
                Bc = 1u;
                Dm &= first;
                Im &= first;
                Sx = Sx && L == 0u;
                nSurv = (uint32_t)__popc(Dm) + (uint32_t)__popc(Im) + (Sx ? 1u : 0u);
            }
            const bool contM1 = node && L >= Bc;
            // cannot happen (the reserve rule above; tests/text_model.py): flagged, not handled
            bad = bad || (node && nSurv && sp + nSurv + (contM1 ? 1u : 0u) - 1u > a.stackCap);

            // ---- children as stack entries (x = span, y = meta). Per step:
            // extending by n symbols adds n << 16 (right) or -n (left) to the
            // span, one mad; a child's side memory is its operation on the
            // extension side (MS once k forced matches follow it), the other
            // side keeps its memory — except at pos 0, where the first
            // operation sets both (for chain node i > 0 that was a match)
            const int extMul = r0 ? 65536 : -1;
            auto extend = [&](uint32_t span, uint32_t n) -> uint32_t { return span + (uint32_t)((int)n * extMul); };
            const uint32_t shMine = r0 ? 22u : 20u, shOther = r0 ? 20u : 22u;
            const uint32_t otherKept = pos ? (r0 ? lastL : lastR) : (uint32_t)OP_MS;
            auto metaAt = [&](uint32_t i, uint32_t op, uint32_t k) -> uint32_t {
                const uint32_t mine = k ? (uint32_t)OP_MS : op;
                const uint32_t other = (pos == 0u && i == 0u) ? op : otherKept;
                return (mine << shMine) | (other << shOther);
            };
            const uint32_t e1 = (e + 1u) << 16;
            // forced matches after an error child whose run starts at chain node ii
            const uint32_t kEnd = kidsF ? run0 : 0u;
            const uint2 cM = make_uint2(extend(cur.x, Bc), (pos + Bc) | (e << 16) | metaAt(Bc, OP_MS, 0u));
            if (nSurv) {  // the surviving error children; the last one stays in registers
                uint32_t spw = sp;
                uint2 pend = cM;
                bool hasPend = contM1;
                // one loop over all of them — D at chain node i (bit i), I at i
                // (bit 32 + i), S at L (bit 63), in that order — so the wave
                // runs max(nSurv) iterations rather than one loop per kind
                uint64_t sv = (uint64_t)Dm | ((uint64_t)Im << 32) | (Sx ? 1ull << 63 : 0ull);
                while (sv) {
                    const uint32_t j = (uint32_t)__builtin_ctzll(sv);
                    sv &= sv - 1ull;
                    const bool isS = j == 63u, isD = j < 32u, isI = !isD && !isS;
                    const uint32_t i = isS ? L : (j & 31u);
                    const uint32_t ii = i + (isD ? 0u : 1u);  // chain node where its forced run starts
                    const uint32_t k = ii < kEnd ? min(kEnd - ii, 7u) : 0u;
                    const uint32_t op = isD ? (uint32_t)OP_D : (isI ? (uint32_t)OP_I : (uint32_t)OP_MS);
                    const uint2 v = make_uint2(extend(cur.x, i + k + (isI ? 0u : 1u)), (pos + ii + k) | e1 | metaAt(i, op, k));
                    if (hasPend) stackPut(min(spw++, a.stackCap - 1u), pend);
                    pend = v;
                    hasPend = true;
                }
                sp = min(spw, a.stackCap);
                cur = pend;
            } else if (node && contM1) {
                cur = cM;
            }

            if (atLeaf) { leaf = true; leafStart = xo; leafE = e; }
            have = live ? node && (nSurv || contM1) : have;
            if (COUNT) {
                cNodes += forced ? 0u : (node ? NN : 0u);
                cCmp += (node && forced) ? 1u : 0u;
                cSteps += node ? 1u : 0u;
            }
        }
        if (COUNT) {
            const uint64_t t1 = clock64();
            cyStep += t1 - t0;
            t0 = t1;
        }
        {
            uint32_t s;
            if (hitSlots.take(leaf, lane, ltMask, a.hitCount, s) && leaf) {
                if (s < a.hitCap) {
                    a.hits[s] = make_uint4(pid, wb + leafStart, 1u, leafE | kPosKnown);
                    // the hit's row ranked in its query's segment (a.qcnt,
                    // the FM phase's counts): the atomic's result is stored
                    // at the lane's next emission, so that its round trip
                    // overlaps the micro-steps in between (kLocate then
                    // places the hit without an atomic of its own)
                    if (rankSlot != ~0u) a.rank[rankSlot] = rankVal;
                    rankVal = atomicAdd(a.qcnt + pid, 1u);
                    rankSlot = s;
                } else {
                    atomicOr(a.flags, 2u);
                }
                ++filled;
            }
        }
        if (COUNT) cyEmit += clock64() - t0;
        if (kProbe && a.probe) {
            const uint64_t pw2 = wall_clock64();
            if (qDone) { pwPostA += pw1 - pw0; pwPostB += pw2 - pw1; }
            else { pwPreA += pw1 - pw0; pwPreB += pw2 - pw1; }
        }
    }
    if (kProbe && a.probe && a.isFirst && lane == 0) {
        const uint64_t wEnd = wall_clock64(), w0 = wBorn[threadIdx.x >> 6], wd = wDrain[threadIdx.x >> 6];
        atomicMin(a.counters + 33, (unsigned long long)w0);
        atomicMax(a.counters + 34, (unsigned long long)w0);
        atomicMax(a.counters + 35, (unsigned long long)wEnd);
        atomicAdd(a.counters + 36, (unsigned long long)(wEnd - w0));
        atomicMin(a.counters + 37, (unsigned long long)wEnd);
        if (wd) {
            atomicMin(a.counters + 38, (unsigned long long)wd);
            atomicMax(a.counters + 39, (unsigned long long)wd);
            atomicAdd(a.counters + 30, (unsigned long long)(wEnd - wd));
            atomicAdd(a.counters + 31, 1ull);
        }
        atomicAdd(a.counters + 40, (unsigned long long)pIterPre);
        atomicAdd(a.counters + 41, (unsigned long long)pActPre);
        atomicAdd(a.counters + 42, (unsigned long long)pIterPost);
        atomicAdd(a.counters + 43, (unsigned long long)pActPost);
        atomicAdd(a.counters + 46, (unsigned long long)pwPreA);
        atomicAdd(a.counters + 47, (unsigned long long)pwPreB);
        atomicAdd(a.counters + 48, (unsigned long long)pwPostA);
        atomicAdd(a.counters + 49, (unsigned long long)pwPostB);
    }
    hitSlots.close(lane, a.hits, a.hitCap);
    if (rankSlot != ~0u) a.rank[rankSlot] = rankVal;
    if (filled) atomicAdd(a.filled, filled);  // per-lane counts
    if (__any(bad) && lane == 0) atomicOr(a.flags, 16u);
    if (COUNT) {
        atomicAdd(a.counters + 5, (unsigned long long)cNodes);
        if (lane == 0) {
            atomicAdd(a.counters + 8, (unsigned long long)tIter);
            atomicAdd(a.counters + 9, (unsigned long long)tActive);
            atomicAdd(a.counters + 10, (unsigned long long)tRefill);
            atomicAdd(a.counters + 11, (unsigned long long)cyRefill);
            atomicAdd(a.counters + 12, (unsigned long long)cyStep);
            atomicAdd(a.counters + 13, (unsigned long long)cyEmit);
        }
        atomicAdd(a.counters + 14, (unsigned long long)cCmp);
        atomicAdd(a.counters + 15, (unsigned long long)cSteps);
        if (cSteal) atomicAdd(a.counters + 45, (unsigned long long)cSteal);
    }
}

// ================================================================ locate ====

// Segment tiers: <= kSmallSeg rows sorted in a lane's registers,
// <= kMediumSeg by a wave (one key per lane, bitonic over shuffles), longer
// ones by the segmented radix sort.
constexpr uint32_t kSmallSeg = 8;
constexpr uint32_t kMediumSeg = 64;
// long segments of <= kLdsSeg rows: one workgroup each, bitonic sort in 16 KB
// of LDS (kSortBigLds); longer ones ("huge"): the segmented radix sort
constexpr uint32_t kLdsSeg = 2048;

// Exclusive scan of the per-query row counts (n = queries + 1 entries, the
// last one 0) into u64 segment offsets, reduce-then-scan over tiles of
// kScanTile: no inter-block waiting, so it keeps its pace next to the
// persistent search kernels. The tile pass also lists the long segments
// (> kMediumSeg rows; one global atomic per tile).
constexpr uint32_t kScanTile = 4096;

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint64_t blockExclusiveScan(uint64_t v, uint64_t& total, uint64_t* wsum) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint64_t pre = 0;
    total = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint64_t t = wsum[i];
        pre += i < w ? t : 0;
        total += t;
    }
    __syncthreads();
    return pre + x - v;
}

__global__ __launch_bounds__(256) void kTileSums(const uint32_t* __restrict__ cnt, uint32_t n,
                                                uint64_t* __restrict__ partial) {
    __shared__ uint64_t wsum[4];
    const uint32_t base = blockIdx.x * kScanTile;
    uint64_t acc = 0;
    for (uint32_t i = threadIdx.x; i < kScanTile && base + i < n; i += 256) acc += cnt[base + i];
    for (uint32_t off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
    if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void kScanPartials(uint64_t* __restrict__ partial, uint32_t ntiles) {
    __shared__ uint64_t wsum[4];
    uint64_t carry = 0;
    for (uint32_t b = 0; b < ntiles; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? partial[i] : 0;
        uint64_t tot;
        const uint64_t ex = blockExclusiveScan(v, tot, wsum);
        if (i < ntiles) partial[i] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void kScanTiles(uint32_t* __restrict__ cnt, uint32_t n,
                                                 const uint64_t* __restrict__ partial, uint64_t* __restrict__ off,
                                                 uint32_t* __restrict__ list, uint32_t* __restrict__ nlist,
                                                 uint32_t* __restrict__ huge, uint32_t* __restrict__ nhuge) {
    __shared__ uint64_t wsum[4];
    __shared__ uint32_t llist[kScanTile];
    __shared__ uint32_t lcnt, lbase;
    const uint32_t lane = threadIdx.x & 63u;
    if (threadIdx.x == 0) lcnt = 0;
    const uint32_t base = blockIdx.x * kScanTile;
    uint64_t carry = partial[blockIdx.x];
    for (uint32_t c = 0; c < kScanTile; c += 256) {  // uniform trip count: block scans inside
        const uint32_t i = base + c + threadIdx.x;
        const uint32_t v = i < n ? cnt[i] : 0u;
        if (v) cnt[i] = 0u;  // zero again for the next batch
        uint64_t tot;
        const uint64_t ex = blockExclusiveScan(v, tot, wsum);
        if (i < n) off[i] = carry + ex;
        carry += tot;
        const uint64_t m = __ballot(v > kMediumSeg);
        if (m) {
            uint32_t wb = 0;
            const int leader = __ffsll((long long)m) - 1;
            if ((int)lane == leader) wb = atomicAdd(&lcnt, (uint32_t)__popcll(m));
            wb = __shfl(wb, leader);
            if (v > kMediumSeg) llist[wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
            if (v > kLdsSeg) huge[atomicAdd(nhuge, 1u)] = i;  // rare: past the LDS sort (kSortBigLds)
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) lbase = lcnt ? atomicAdd(nlist, lcnt) : 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < lcnt; i += 256) list[lbase + i] = llist[i];
}

// One lane per reported cursor: locate every row of [lb, lb+len) into the
// query's segment [qoff[qid], qoff[qid+1]) of the key array (key = text
// position << 4 | e), from the slot the search kernel ranked it at (rank).
template <bool COUNT>
__global__ __launch_bounds__(256) void kLocate(LocateArgs a) {
    uint64_t steps = 0;
    for (uint64_t h = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; h < a.nhits;
         h += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 hit = a.hits[h];
        if (hit.z == 0) continue;  // reserved hole
        const uint64_t e = hit.w & 0xFu;
        const uint64_t out = a.qoff[hit.x] + a.rank[h];
        if (hit.w & kPosKnown) {  // resolved by the text phase, ranked where it was written
            a.keys[out] = ((uint64_t)hit.y << 4) | e;
            continue;
        }
        if (a.useSA) {  // full SA resident: one read per row
            for (uint32_t j = 0; j < hit.z; ++j) a.keys[out + j] = ((uint64_t)a.sa[hit.y + j] << 4) | e;
            continue;
        }
        for (uint32_t j = 0; j < hit.z; ++j) {  // fmc::LocateLinear: LF walk to a sample
            uint32_t row = hit.y + j;
            uint32_t st = 0;
            uint64_t gpos = 0;
            for (;;) {
                const uint4* q = reinterpret_cast<const uint4*>(a.occF + (row >> 6));
                const uint4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
                const uint32_t o = row & 63u;
                const uint64_t sampled = (uint64_t)a3.x | ((uint64_t)a3.y << 32);
                if ((sampled >> o) & 1ull) {
                    const uint32_t k = a1.y + (uint32_t)__popcll(sampled & lowMask(o));
                    gpos = (uint64_t)a.samples[k] + st;
                    break;
                }
                const uint64_t p[3] = {(uint64_t)a1.z | ((uint64_t)a1.w << 32),
                                       (uint64_t)a2.x | ((uint64_t)a2.y << 32),
                                       (uint64_t)a2.z | ((uint64_t)a2.w << 32)};
                const uint32_t c = symAt(p, o);
                if (c == 0 || st >= a.rate) {  // cannot happen on a well-formed index
                    atomicOr(a.flags, 4u);
                    break;
                }
                const uint32_t cnt[5] = {a0.x, a0.y, a0.z, a0.w, a1.x};
                row = a.C[c] + pick5(cnt, c - 1) + (uint32_t)__popcll(symMask(p, c) & lowMask(o));
                ++st;
            }
            if (COUNT) steps += st;
            a.keys[out + j] = (gpos << 4) | e;
        }
    }
    if (COUNT && steps) atomicAdd(a.counters, (unsigned long long)steps);
}

__device__ __forceinline__ sahara_hit decodeKey(uint64_t k, uint64_t qid, const uint64_t* __restrict__ starts,
                                                uint32_t nrec) {
    const uint64_t gpos = k >> 4;
    uint32_t lo = 0, hi = nrec;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= gpos) lo = mid; else hi = mid;
    }
    sahara_hit h;
    h.qid = qid;
    h.seq_id = lo;
    h.err = (uint32_t)(k & 15u);
    h.pos = gpos - starts[lo];
    return h;
}

__device__ __forceinline__ void cswap(uint64_t& a, uint64_t& b) {
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Sort + decode, one workgroup per 256 consecutive queries. Their segments
// are one contiguous key range; when it fits kTileKeys (the common case: ~1.3
// rows per query) it is staged in LDS by coalesced loads, every segment is
// sorted there, and the decoded hits leave as one coalesced run of 24-B
// records. Per segment: <= kSmallSeg rows sorted in the lane's registers
// (odd-even transposition, padded with ~0); medium ones by the wave, one key
// per lane, bitonic over shuffles; long ones are left to the segmented radix
// sort (kDecodeBig). Record starts sit in LDS for texts of <= kLdsStarts
// records, so a decode's binary search waits on no global loads. A range
// larger than the tile takes the same tiers straight from global memory.
constexpr uint32_t kTileKeys = 1024;
constexpr uint32_t kLdsStarts = 256;
constexpr uint16_t kSkipRow = 0xFFFFu;

__global__ __launch_bounds__(256) void kSortDecode(const uint64_t* __restrict__ keys,
                                                  const uint64_t* __restrict__ qoff, uint32_t nq, uint64_t qidBase,
                                                  const uint64_t* __restrict__ starts, uint32_t nrec,
                                                  sahara_hit* __restrict__ out) {
    __shared__ uint64_t sk[kTileKeys];
    __shared__ uint64_t soff[257];
    __shared__ uint64_t sst[kLdsStarts];
    __shared__ uint16_t sq[kTileKeys];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const bool ldsStarts = nrec <= kLdsStarts;
    if (ldsStarts)
        for (uint32_t i = t; i < nrec; i += 256) sst[i] = starts[i];
    auto decode = [&](uint64_t k, uint64_t qid) {
        const uint64_t gpos = k >> 4;
        uint32_t lo = 0, hi = nrec;
        uint64_t s0 = 0;
        if (ldsStarts) {
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (sst[mid] <= gpos) lo = mid; else hi = mid;
            }
            s0 = sst[lo];
        } else {
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (starts[mid] <= gpos) lo = mid; else hi = mid;
            }
            s0 = starts[lo];
        }
        sahara_hit h;
        h.qid = qid;
        h.seq_id = lo;
        h.err = (uint32_t)(k & 15u);
        h.pos = gpos - s0;
        return h;
    };
    for (uint32_t q0 = blockIdx.x * 256u; q0 < nq; q0 += gridDim.x * 256u) {
        const uint32_t q = q0 + t;
        soff[t] = qoff[q < nq ? q : nq];
        if (t == 0) soff[256] = qoff[q0 + 256u < nq ? q0 + 256u : nq];
        __syncthreads();
        const uint64_t base = soff[0], R = soff[256] - base;
        const uint64_t b = soff[t];
        const uint32_t n = q < nq ? (uint32_t)(soff[t + 1] - b) : 0u;
        if (R <= kTileKeys) {  // block-uniform
            for (uint32_t i = t; i < (uint32_t)R; i += 256) sk[i] = keys[base + i];
            __syncthreads();
            const uint32_t lb = (uint32_t)(b - base);
            if (n && n <= kSmallSeg) {
                uint64_t v[kSmallSeg];
#pragma unroll
                for (uint32_t i = 0; i < kSmallSeg; ++i) v[i] = i < n ? sk[lb + i] : ~0ull;
#pragma unroll
                for (uint32_t r = 0; r < kSmallSeg; ++r) {
                    if (r >= n) break;
#pragma unroll
                    for (uint32_t i = r & 1u; i + 1 < kSmallSeg; i += 2) cswap(v[i], v[i + 1]);
                }
#pragma unroll
                for (uint32_t i = 0; i < kSmallSeg; ++i)
                    if (i < n) {
                        sk[lb + i] = v[i];
                        sq[lb + i] = (uint16_t)t;
                    }
            } else if (n > kMediumSeg) {
                for (uint32_t i = 0; i < n; ++i) sq[lb + i] = kSkipRow;  // the radix path decodes it
            }
            uint64_t med = __ballot(n > kSmallSeg && n <= kMediumSeg);
            while (med) {
                const int src = __ffsll((long long)med) - 1;
                med &= med - 1;
                const uint32_t sn = (uint32_t)__shfl((int)n, src), slb = (uint32_t)__shfl((int)lb, src);
                uint64_t v = lane < sn ? sk[slb + lane] : ~0ull;
#pragma unroll
                for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
                    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                        const uint64_t o = __shfl_xor(v, j);
                        const bool keepMin = ((lane & j) == 0) == ((lane & k) == 0);
                        v = keepMin ? (v < o ? v : o) : (v < o ? o : v);
                    }
                }
                if (lane < sn) {
                    sk[slb + lane] = v;
                    sq[slb + lane] = (uint16_t)((t & ~63u) + (uint32_t)src);
                }
            }
            __syncthreads();
            for (uint32_t i = t; i < (uint32_t)R; i += 256) {
                const uint32_t lq = sq[i];
                if (lq != kSkipRow) out[base + i] = decode(sk[i], qidBase + q0 + lq);
            }
            __syncthreads();  // soff, sk, sq are reused by the next range
            continue;
        }
        __syncthreads();  // soff is reused by the next range
        if (n && n <= kSmallSeg) {
            uint64_t v[kSmallSeg];
#pragma unroll
            for (uint32_t i = 0; i < kSmallSeg; ++i) v[i] = i < n ? keys[b + i] : ~0ull;
            // n rounds sort the n keys (the ~0 padding never moves)
#pragma unroll
            for (uint32_t r = 0; r < kSmallSeg; ++r) {
                if (r >= n) break;
#pragma unroll
                for (uint32_t i = r & 1u; i + 1 < kSmallSeg; i += 2) cswap(v[i], v[i + 1]);
            }
#pragma unroll
            for (uint32_t i = 0; i < kSmallSeg; ++i)
                if (i < n) out[b + i] = decode(v[i], qidBase + q);
        }
        uint64_t med = __ballot(n > kSmallSeg && n <= kMediumSeg);
        while (med) {
            const int src = __ffsll((long long)med) - 1;
            med &= med - 1;
            const uint32_t sqid = (uint32_t)__shfl((int)q, src), sn = (uint32_t)__shfl((int)n, src);
            const uint64_t sb = __shfl(b, src);
            uint64_t v = lane < sn ? keys[sb + lane] : ~0ull;
#pragma unroll
            for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    const uint64_t o = __shfl_xor(v, j);
                    const bool keepMin = ((lane & j) == 0) == ((lane & k) == 0);
                    v = keepMin ? (v < o ? v : o) : (v < o ? o : v);
                }
            }
            if (lane < sn) out[sb + lane] = decode(v, qidBase + sqid);
        }
    }
}

// One workgroup per long segment (already sorted): decode.
__global__ __launch_bounds__(256) void kDecodeBig(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ qoff,
                                                 const uint32_t* __restrict__ big, uint32_t nbig, uint64_t qidBase,
                                                 const uint64_t* __restrict__ starts, uint32_t nrec,
                                                 sahara_hit* __restrict__ out) {
    for (uint32_t s = blockIdx.x; s < nbig; s += gridDim.x) {
        const uint32_t q = big[s];
        const uint64_t b = qoff[q], e = qoff[q + 1];
        for (uint64_t i = b + threadIdx.x; i < e; i += blockDim.x) out[i] = decodeKey(keys[i], qidBase + q, starts, nrec);
    }
}

// Long segments (kMediumSeg < rows <= kLdsSeg): one workgroup per segment,
// keys padded to a power of two with ~0 in LDS, bitonic sort, decoded hits
// written in order. 16 KB of LDS and no scratch in HBM: it fits beside the
// text phase's workgroups, where rocPRIM's segmented radix sort (whose blocks
// need more LDS than the text phase leaves free) waited for the text launch
// to drain, up to 1.3 ms per batch at C3 (profiles/r03_v5_c3_timeline.txt).
__global__ __launch_bounds__(256) void kSortBigLds(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ qoff,
                                                  const uint32_t* __restrict__ big, uint32_t nbig, uint64_t qidBase,
                                                  const uint64_t* __restrict__ starts, uint32_t nrec,
                                                  sahara_hit* __restrict__ out) {
    __shared__ uint64_t K[kLdsSeg];
    for (uint32_t s = blockIdx.x; s < nbig; s += gridDim.x) {
        const uint32_t q = big[s];
        const uint64_t b = qoff[q], e = qoff[q + 1];
        const uint32_t n = (uint32_t)(e - b);
        if (n > kLdsSeg) continue;  // a huge segment: the radix sort path (block-uniform)
        uint32_t P = 1;
        while (P < n) P <<= 1;
        for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) K[i] = i < n ? keys[b + i] : ~0ull;
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
                    const uint32_t p = i ^ j;
                    if (p > i) {
                        const uint64_t x = K[i], y = K[p];
                        const bool up = (i & k) == 0;
                        if ((x > y) == up) {
                            K[i] = y;
                            K[p] = x;
                        }
                    }
                }
                __syncthreads();
            }
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) out[b + i] = decodeKey(K[i], qidBase + q, starts, nrec);
        __syncthreads();
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

__global__ void kDigest(const sahara_hit* __restrict__ h, uint64_t n, unsigned long long* out) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        acc += mix64(h[i].qid * 0x9E3779B97F4A7C15ull ^ mix64(((uint64_t)h[i].seq_id << 40) ^ (h[i].pos << 4) ^ h[i].err));
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, (unsigned long long)acc);
}

// Hit records into a caller's device buffer with qids shifted by qidOffset
// (rank-local -> global qids before a gather across ranks).
__global__ void kCopyHits(const sahara_hit* __restrict__ h, uint64_t n, uint64_t qidOffset,
                          sahara_hit* __restrict__ dst) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        sahara_hit r = h[i];
        r.qid += qidOffset;
        dst[i] = r;
    }
}

// pattern bytes (one symbol per byte) -> 4-bit words, patWords per pattern
// Also validates the ranks (ivs::verify_rank, search.cpp:118-120): *bad != 0
// if any is 0 or >= sigma.
__global__ void kPackPatterns(const uint8_t* __restrict__ src, uint64_t npat, uint32_t m, uint32_t patWords,
                              uint32_t sigma, uint32_t* __restrict__ dst, uint32_t* __restrict__ bad) {
    const uint64_t total = npat * patWords;
    bool invalid = false;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = i / patWords;
        const uint32_t w = (uint32_t)(i - p * patWords);
        uint32_t v = 0;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t q = w * 8 + j;
            if (q < m) {
                const uint32_t r = src[p * m + q];
                invalid |= r == 0 || r >= sigma;
                v |= (r & 0xFu) << (4 * j);
            }
        }
        dst[i] = v;
    }
    if (__any(invalid) && (threadIdx.x & 63u) == 0) atomicOr(bad, 1u);
}

// pattern bytes -> 3-bit-plane blocks of 32 symbols (device_index.h),
// patBlocks per pattern, zero past m (the text phase's layout)
__global__ void kPackPatterns3(const uint8_t* __restrict__ src, uint64_t npat, uint32_t m, uint32_t patBlocks,
                               uint4* __restrict__ dst) {
    const uint64_t total = npat * patBlocks;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = i / patBlocks;
        const uint32_t b = (uint32_t)(i - p * patBlocks);
        uint32_t p0 = 0, p1 = 0, p2 = 0;
        for (uint32_t j = 0; j < 32; ++j) {
            const uint32_t q = b * 32 + j;
            if (q < m) {
                const uint32_t r = src[p * m + q];
                p0 |= (r & 1u) << j;
                p1 |= ((r >> 1) & 1u) << j;
                p2 |= ((r >> 2) & 1u) << j;
            }
        }
        dst[i] = make_uint4(p0, p1, p2, 0u);
    }
}

struct SegOff {  // begin (d = 0) / end (d = 1) of a listed query's segment
    const uint64_t* qoff;
    uint32_t d;
    __host__ __device__ uint32_t operator()(const uint32_t& q) const { return (uint32_t)qoff[q + d]; }
};

template <int SIGMA>
void launchFMT(const SearchArgs& a, bool edit, bool count, dim3 grid, size_t lds, hipStream_t st) {
    if (edit) {
        if (count) hipLaunchKernelGGL((kSearchFM<SIGMA, true, true>), grid, dim3(256), lds, st, a);
        else       hipLaunchKernelGGL((kSearchFM<SIGMA, true, false>), grid, dim3(256), lds, st, a);
    } else {
        if (count) hipLaunchKernelGGL((kSearchFM<SIGMA, false, true>), grid, dim3(256), lds, st, a);
        else       hipLaunchKernelGGL((kSearchFM<SIGMA, false, false>), grid, dim3(256), lds, st, a);
    }
}



}  // namespace

// the compile-time shape matching a launch (0: the generic kernel)
int textShapeOf(uint32_t winBlocks, uint32_t patBlocks, bool exactWindow) {
    for (int shape = 1; shape <= 2; ++shape) {
        const TextShape t = textShape(shape);
        if (winBlocks == t.win && patBlocks == t.pat && exactWindow == t.exact) return shape;
    }
    return 0;
}

int searchBlocksPerCU(uint32_t sigma, bool edit, size_t lds) {
    int b = 0;
    const void* f;
    if (sigma == 5) f = edit ? (const void*)kSearchFM<5, true, false> : (const void*)kSearchFM<5, false, false>;
    else            f = edit ? (const void*)kSearchFM<6, true, false> : (const void*)kSearchFM<6, false, false>;
    SH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, 256, lds));
    return b < 1 ? 1 : b;
}

template <int SIGMA>
const void* textBatchKernelOf(bool edit, bool count, int shape) {
#define SH_TB(S)                                                                                         \
    if (shape == S)                                                                                      \
        return edit ? (count ? (const void*)kSearchTextBatch<SIGMA, true, true, S>                       \
                             : (const void*)kSearchTextBatch<SIGMA, true, false, S>)                     \
                    : (count ? (const void*)kSearchTextBatch<SIGMA, false, true, S>                      \
                             : (const void*)kSearchTextBatch<SIGMA, false, false, S>);
    SH_TB(1)
    SH_TB(2)
    SH_TB(0)
#undef SH_TB
    return nullptr;
}

int textBlocksPerCU(uint32_t sigma, bool edit, bool count, int shape, size_t lds) {
    // (the variant that is launched: its registers differ by shape and count mode)
    int b = 0;
    const void* f = sigma == 5 ? textBatchKernelOf<5>(edit, count, shape) : textBatchKernelOf<6>(edit, count, shape);
    SH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, 256, lds));
    return b;
}

void launchSearch(const SearchArgs& a, uint32_t sigma, bool edit, bool count, uint32_t blocks, size_t lds,
                  hipStream_t st) {
    if (sigma == 5) launchFMT<5>(a, edit, count, dim3(blocks), lds, st);
    else            launchFMT<6>(a, edit, count, dim3(blocks), lds, st);
    SH_HIP(hipGetLastError());
}

template <int SIGMA, int SHAPE>
void launchTextBatchShaped(const TextBatchArgs& a, bool edit, bool count, dim3 grid, size_t lds, hipStream_t st) {
    if (edit) {
        if (count) hipLaunchKernelGGL((kSearchTextBatch<SIGMA, true, true, SHAPE>), grid, dim3(256), lds, st, a);
        else       hipLaunchKernelGGL((kSearchTextBatch<SIGMA, true, false, SHAPE>), grid, dim3(256), lds, st, a);
    } else {
        if (count) hipLaunchKernelGGL((kSearchTextBatch<SIGMA, false, true, SHAPE>), grid, dim3(256), lds, st, a);
        else       hipLaunchKernelGGL((kSearchTextBatch<SIGMA, false, false, SHAPE>), grid, dim3(256), lds, st, a);
    }
}

template <int SIGMA>
void launchTextBatchT(const TextBatchArgs& a, bool edit, bool count, dim3 grid, size_t lds, hipStream_t st) {
    const int shape = textShapeOf(a.winBlocks, a.patBlocks, a.exactWindow != 0u);
    if (shape == 1) launchTextBatchShaped<SIGMA, 1>(a, edit, count, grid, lds, st);
    else if (shape == 2) launchTextBatchShaped<SIGMA, 2>(a, edit, count, grid, lds, st);
    else launchTextBatchShaped<SIGMA, 0>(a, edit, count, grid, lds, st);
}

void launchTextBatch(const TextBatchArgs& a, uint32_t sigma, bool edit, bool count, uint32_t blocks, size_t lds,
                     hipStream_t st) {
    if (sigma == 5) launchTextBatchT<5>(a, edit, count, dim3(blocks), lds, st);
    else            launchTextBatchT<6>(a, edit, count, dim3(blocks), lds, st);
    SH_HIP(hipGetLastError());
}

void launchSeeds(const SeedArgs& a, uint32_t sigma, uint32_t blocks, hipStream_t st) {
    if (sigma == 5) hipLaunchKernelGGL((kSeedItems<5>), dim3(blocks), dim3(256), 0, st, a);
    else            hipLaunchKernelGGL((kSeedItems<6>), dim3(blocks), dim3(256), 0, st, a);
    SH_HIP(hipGetLastError());
}

// Host upload format -> one byte per symbol: byte i of `nib` holds symbols 2i
// (low nibble) and 2i + 1 (high nibble). A thread expands 8 bytes into 16.
__global__ void kUnpackNibbles(const uint8_t* __restrict__ nib, uint8_t* __restrict__ dst, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w * 16 < n; w += stride) {
        if (w * 16 + 16 <= n) {
            const uint64_t x = *reinterpret_cast<const uint64_t*>(nib + w * 8);
            uint32_t o[4];
            for (int q = 0; q < 4; ++q) {
                const uint32_t b = (uint32_t)(x >> (16 * q));   // two packed bytes -> four symbols
                o[q] = (b & 0xFu) | ((b >> 4) & 0xFu) << 8 | ((b >> 8) & 0xFu) << 16 | ((b >> 12) & 0xFu) << 24;
            }
            *reinterpret_cast<uint4*>(dst + w * 16) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            for (uint64_t i = w * 16; i < n; ++i) dst[i] = (nib[i >> 1] >> ((i & 1) * 4)) & 0xFu;
        }
    }
}

void launchUnpackNibbles(const uint8_t* nib, uint8_t* dst, uint64_t n, hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>((n / 16 + 256) / 256, 65536);
    hipLaunchKernelGGL(kUnpackNibbles, dim3((unsigned)blocks), dim3(256), 0, st, nib, dst, n);
    SH_HIP(hipGetLastError());
}

// Multi-part index (capi.cpp run): a part's hits with its first global
// record id added to seq_id, appended to the hits of the parts before it.
__global__ void kOffsetSeq(const sahara_hit* __restrict__ in, uint64_t n, uint32_t rec0, sahara_hit* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        sahara_hit h = in[i];
        h.seq_id += rec0;
        out[i] = h;
    }
}

void launchOffsetSeq(const sahara_hit* in, uint64_t n, uint64_t rec0, sahara_hit* out, hipStream_t st) {
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(kOffsetSeq, dim3((unsigned)blocks), dim3(256), 0, st, in, n, (uint32_t)rec0, out);
    SH_HIP(hipGetLastError());
}

__global__ void kQidKeys(const sahara_hit* __restrict__ h, uint64_t n, uint64_t* __restrict__ key,
                         uint32_t* __restrict__ idx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        key[i] = h[i].qid;
        idx[i] = (uint32_t)i;
    }
}

__global__ void kGatherHits(const sahara_hit* __restrict__ in, const uint32_t* __restrict__ idx, uint64_t n,
                            sahara_hit* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[idx[i]];
}

// --max_hits n on the device (search_n, search.cpp:228,231; the policy U6 of
// include/sahara_hip.h): per query, of its hits in canonical order, the n
// distinct (seq_id, pos) with the fewest errors (each once, with its minimum
// e: the first of its run), ties by (seq_id, pos). One thread per query: the
// plan counts the distinct positions per error count and fixes the error
// threshold e* and how many at e* are kept (quota); the write keeps, in
// order, every first-of-run below e* and the first `quota` at e*.
struct LimitPlan { uint32_t eStar, quota, kept; };
__device__ __forceinline__ LimitPlan limitPlan(const sahara_hit* __restrict__ h, uint64_t b, uint64_t e, uint32_t n) {
    uint32_t hist[16];
#pragma unroll
    for (uint32_t x = 0; x < 16; ++x) hist[x] = 0;
    uint32_t distinct = 0, ps = 0xFFFFFFFFu;
    uint64_t pp = ~0ull;
    for (uint64_t i = b; i < e; ++i) {
        const sahara_hit x = h[i];
        if (x.seq_id != ps || x.pos != pp) {
            ++distinct;
#pragma unroll
            for (uint32_t v = 0; v < 16; ++v) hist[v] += x.err == v ? 1u : 0u;
            ps = x.seq_id;
            pp = x.pos;
        }
    }
    if (distinct <= n) return {16u, 0u, distinct};
    uint32_t cum = 0;
#pragma unroll
    for (uint32_t v = 0; v < 16; ++v) {
        if (cum < n && cum + hist[v] >= n) return {v, n - cum, n};
        cum += hist[v];
    }
    return {16u, 0u, distinct};  // unreachable: the histogram sums to distinct > n
}

__global__ void kLimitCount(const sahara_hit* __restrict__ h, const uint64_t* __restrict__ qoff, uint32_t nq,
                            uint32_t n, uint32_t* __restrict__ kcnt) {
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q <= nq; q += gridDim.x * blockDim.x)
        kcnt[q] = q < nq ? limitPlan(h, qoff[q], qoff[q + 1], n).kept : 0u;
}

__global__ void kLimitWrite(const sahara_hit* __restrict__ h, const uint64_t* __restrict__ qoff, uint32_t nq,
                            uint32_t n, const uint64_t* __restrict__ koff, sahara_hit* __restrict__ dst) {
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
        const uint64_t b = qoff[q], e = qoff[q + 1];
        const LimitPlan P = limitPlan(h, b, e, n);
        uint64_t w = koff[q];
        uint32_t used = 0, ps = 0xFFFFFFFFu;
        uint64_t pp = ~0ull;
        for (uint64_t i = b; i < e; ++i) {
            const sahara_hit x = h[i];
            if (x.seq_id == ps && x.pos == pp) continue;
            ps = x.seq_id;
            pp = x.pos;
            const bool keep = x.err < P.eStar || (x.err == P.eStar && used < P.quota);
            used += x.err == P.eStar && keep ? 1u : 0u;
            if (keep) dst[w++] = x;
        }
    }
}

// Applies --max_hits n to one batch's hits (out, rows; per-query segments
// qoff[0..nq]) in place; returns the rows kept. Host-synchronous (the kept
// total sizes the rest of the batch's chain): read back through hostKept,
// 8 B of pinned memory.
uint64_t limitBatch(sahara_hit* out, uint64_t rows, const uint64_t* qoff, uint32_t nq, uint32_t n,
                    DevBuf<uint32_t>& kcnt, DevBuf<uint64_t>& koff, DevBuf<sahara_hit>& buf, DevBuf<char>& tmp,
                    uint64_t* hostKept, hipStream_t st) {
    if (rows == 0 || nq == 0) return rows;
    kcnt.reserve((size_t)nq + 1);
    koff.reserve((size_t)nq + 1);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((nq + 256) / 256, 16384));
    hipLaunchKernelGGL(kLimitCount, dim3(blocks), dim3(256), 0, st, out, qoff, nq, n, kcnt.ptr);
    SH_HIP(hipGetLastError());
    size_t bytes = 0;
    SH_HIP(rocprim::exclusive_scan(nullptr, bytes, kcnt.ptr, koff.ptr, (uint64_t)0, (size_t)nq + 1,
                                   rocprim::plus<uint64_t>(), st));
    tmp.reserve(bytes + 256);
    SH_HIP(rocprim::exclusive_scan(tmp.ptr, bytes, kcnt.ptr, koff.ptr, (uint64_t)0, (size_t)nq + 1,
                                   rocprim::plus<uint64_t>(), st));
    SH_HIP(hipMemcpyAsync(hostKept, koff.ptr + nq, 8, hipMemcpyDeviceToHost, st));
    SH_HIP(hipStreamSynchronize(st));
    const uint64_t kept = *hostKept;
    if (kept == rows) return rows;  // nothing to drop in this batch
    buf.reserve(std::max<uint64_t>(kept, 1));
    hipLaunchKernelGGL(kLimitWrite, dim3(blocks), dim3(256), 0, st, out, qoff, nq, n, koff.ptr, buf.ptr);
    SH_HIP(hipGetLastError());
    if (kept) SH_HIP(hipMemcpyAsync(out, buf.ptr, kept * sizeof(sahara_hit), hipMemcpyDeviceToDevice, st));
    return kept;
}

// Stable sort of hit records by qid (rocPRIM's LSD radix sort is stable):
// the parts' hits, each part in canonical order and every part's records
// after the previous part's, come out in canonical (qid, seq_id, pos, err)
// order. Only the bits of qids below nqid are sorted; the key / index
// buffers (B) are the context's, reused across calls.
void sortHitsByQid(const sahara_hit* in, uint64_t n, uint64_t nqid, sahara_hit* out, MergeBufs& B, DevBuf<char>& tmp,
                   hipStream_t st) {
    if (n == 0) return;
    if (n >= (1ull << 32)) throw Error("more than 2^32 hits to merge across index parts");
    B.k0.reserve(n);
    B.k1.reserve(n);
    B.v0.reserve(n);
    B.v1.reserve(n);
    unsigned endBit = 1;
    while (endBit < 64 && (nqid > (1ull << endBit))) ++endBit;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(kQidKeys, dim3((unsigned)blocks), dim3(256), 0, st, in, n, B.k0.ptr, B.v0.ptr);
    SH_HIP(hipGetLastError());
    size_t bytes = 0;
    SH_HIP(rocprim::radix_sort_pairs(nullptr, bytes, B.k0.ptr, B.k1.ptr, B.v0.ptr, B.v1.ptr, (size_t)n, 0, endBit, st));
    tmp.reserve(bytes + 256);
    SH_HIP(rocprim::radix_sort_pairs(tmp.ptr, bytes, B.k0.ptr, B.k1.ptr, B.v0.ptr, B.v1.ptr, (size_t)n, 0, endBit, st));
    hipLaunchKernelGGL(kGatherHits, dim3((unsigned)blocks), dim3(256), 0, st, in, B.v1.ptr, n, out);
    SH_HIP(hipGetLastError());
    SH_HIP(hipStreamSynchronize(st));
}

// sahara_gpu_search's download form of a batch's hits, 8 B instead of 24:
// (qid - qidBase) << 36 | text position << 4 | e (batches < 2^28 queries,
// texts < 2^32, e < 16), expanded back on the host (capi.cpp expandHits).
__global__ void kCompactHits(const sahara_hit* __restrict__ h, uint64_t n, uint64_t qidBase,
                             const uint64_t* __restrict__ starts, uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sahara_hit x = h[i];
        out[i] = ((x.qid - qidBase) << 36) | ((starts[x.seq_id] + x.pos) << 4) | x.err;
    }
}

// `out` may be page-locked host memory: then the kernel's stores are the
// PCIe transfer (posted writes, ~link rate), and a few workgroups (maxBlocks)
// keep it off most CUs.
void launchCompactHits(const sahara_hit* h, uint64_t n, uint64_t qidBase, const uint64_t* starts, uint64_t* out,
                       hipStream_t st, uint32_t maxBlocks) {
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, std::max<uint32_t>(maxBlocks, 1));
    hipLaunchKernelGGL(kCompactHits, dim3((unsigned)blocks), dim3(256), 0, st, h, n, qidBase, starts, out);
    SH_HIP(hipGetLastError());
}

// A streamed 2-bit chunk straight into the search's two pattern forms, with
// no byte pass: 4-bit words (FM phase) and 3-bit-plane blocks (text phase)
// of the patterns [p0, p1). Pattern p is row p, or (rc) read p / 2 and, for
// odd p, its reverse complement (search.cpp:121-123: reversed, codes
// complemented as c ^ 3); read r starts at chunk-local symbol so + (r - r0) * m
// (so < 4: reads given packed start anywhere in a byte).
// `exc` lists the chunk's N positions in ascending order (rank 4). One thread
// per (pattern, 32-symbol block): 64 bits of codes from three word loads,
// even / odd bits gathered into the code planes c0 / c1, then
//   rank bit 0 = ~c0 | c1 (dna5: T = 5) or ~c0 (dna4), bit 1 = c0 ^ c1,
//   bit 2 = c0 & c1, and N = 100.
__device__ __forceinline__ uint32_t evenBits(uint64_t x) {
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    return (uint32_t)(x | (x >> 16));
}
__device__ __forceinline__ uint32_t spreadNibbles(uint32_t x) {  // bit j of 8 -> bit 4j
    x &= 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    return (x | (x << 3)) & 0x11111111u;
}
__global__ void kPackFrom2(const uint8_t* __restrict__ src, uint32_t so, const uint32_t* __restrict__ exc,
                           uint32_t nExc, uint64_t r0, uint64_t p0, uint64_t p1, uint32_t m, uint32_t rc, uint32_t dna5,
                           uint32_t patWords, uint32_t patBlocks, uint32_t* __restrict__ pats,
                           uint4* __restrict__ pats3) {
    const uint64_t total = (p1 - p0) * patBlocks;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = p0 + i / patBlocks;
        const uint32_t b = (uint32_t)(i % patBlocks);
        const uint64_t r = rc ? p >> 1 : p;
        const bool rev = rc && (p & 1u);
        const uint32_t nsym = min(32u, m - 32u * b);
        const uint64_t start = so + (r - r0) * m + (rev ? m - 32u * b - nsym : 32u * b);  // source symbols [start, start + nsym)
        const uint32_t* w = reinterpret_cast<const uint32_t*>(src + (start >> 4) * 4);
        const uint32_t sh = (uint32_t)(start & 15u) * 2u;
        uint64_t v = ((uint64_t)w[1] << 32) | w[0];
        if (sh) v = (v >> sh) | ((uint64_t)w[2] << (64u - sh));
        uint32_t c0 = evenBits(v), c1 = evenBits(v >> 1);
        const uint32_t valid = nsym >= 32u ? 0xFFFFFFFFu : (1u << nsym) - 1u;
        uint32_t nm = 0;
        if (nExc) {
            uint32_t lo = 0, hi = nExc;  // first listed N at or after start
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (exc[mid] < start) lo = mid + 1; else hi = mid;
            }
            for (; lo < nExc && exc[lo] < start + nsym; ++lo) nm |= 1u << (uint32_t)(exc[lo] - start);
        }
        if (rev) {  // symbol q = complement of source symbol nsym - 1 - q
            c0 = ~__builtin_bitreverse32(c0) >> (32u - nsym);
            c1 = ~__builtin_bitreverse32(c1) >> (32u - nsym);
            nm = __builtin_bitreverse32(nm) >> (32u - nsym);
        }
        const uint32_t P0 = ((dna5 ? (~c0 | c1) : ~c0) & ~nm) & valid;
        const uint32_t P1 = ((c0 ^ c1) & ~nm) & valid;
        const uint32_t P2 = ((c0 & c1) | nm) & valid;
        pats3[p * patBlocks + b] = make_uint4(P0, P1, P2, 0u);
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
            const uint32_t wi = 4u * b + t;
            if (wi < patWords)
                pats[p * patWords + wi] = spreadNibbles(P0 >> (8 * t)) | (spreadNibbles(P1 >> (8 * t)) << 1) |
                                          (spreadNibbles(P2 >> (8 * t)) << 2);
        }
    }
}

void launchPackFrom2(const uint8_t* src, uint32_t so, const uint32_t* exc, uint32_t nExc, uint64_t r0, uint64_t p0,
                     uint64_t p1, uint32_t m, bool rc, uint32_t sigma, uint32_t patWords, uint32_t patBlocks,
                     uint32_t* pats, uint4* pats3, hipStream_t st) {
    const uint64_t total = (p1 - p0) * patBlocks;
    if (total == 0) return;
    const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(kPackFrom2, dim3((unsigned)blocks), dim3(256), 0, st, src, so, exc, nExc, r0, p0, p1, m,
                       rc ? 1u : 0u, sigma == 6 ? 1u : 0u, patWords, patBlocks, pats, pats3);
    SH_HIP(hipGetLastError());
}

// Query ingest's reverse-complement interleave (search.cpp:121-127) on the
// device: pattern 2r = read r, 2r + 1 = its reverse complement (A<->T, C<->G,
// N->N; ivs::reverse_complement_rank), for the patterns [2 * r0, pEnd) of the
// reads [r0, r1). One wave per read: lane j copies symbol j and writes its
// complement to position m - 1 - j of the next pattern (coalesced bytes).
__global__ void kInterleaveRC(const uint8_t* __restrict__ reads, uint64_t r0, uint64_t r1, uint32_t m,
                              uint32_t sigma, uint64_t pEnd, uint8_t* __restrict__ pats) {
    const uint32_t comp = sigma == 6 ? 0x142350u : 0x12340u;  // nibble c: complement of rank c (0 past sigma)
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t r = r0 + (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < r1; r += waves) {
        const uint8_t* src = reads + r * m;
        uint8_t* fwd = pats + 2 * r * m;
        uint8_t* rev = fwd + m;
        const bool withRev = 2 * r + 1 < pEnd;
        for (uint32_t j = lane; j < m; j += 64) {
            const uint32_t s = src[j];
            fwd[j] = (uint8_t)s;
            if (withRev) rev[m - 1 - j] = s < 8 ? (uint8_t)((comp >> (4 * s)) & 0xFu) : (uint8_t)0;
        }
    }
}

void launchInterleaveRC(const uint8_t* reads, uint64_t r0, uint64_t r1, uint32_t m, uint32_t sigma, uint64_t pEnd,
                        uint8_t* pats, hipStream_t st) {
    r1 = std::min(r1, (pEnd + 1) / 2);  // reads whose forward pattern is within the limit
    if (r1 <= r0) return;
    const uint64_t blocks = std::min<uint64_t>((r1 - r0 + 3) / 4, 65536);
    hipLaunchKernelGGL(kInterleaveRC, dim3((unsigned)blocks), dim3(256), 0, st, reads, r0, r1, m, sigma, pEnd, pats);
    SH_HIP(hipGetLastError());
}

void launchPackPatterns(const uint8_t* src, uint64_t npat, uint32_t m, uint32_t patWords, uint32_t sigma,
                        uint32_t* dst, uint32_t* bad, hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>((npat * patWords + 255) / 256, 65536);
    hipLaunchKernelGGL(kPackPatterns, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, st, src, npat, m,
                       patWords, sigma, dst, bad);
    SH_HIP(hipGetLastError());
}

void querySegments(uint32_t* qcnt, uint32_t nq, uint64_t* qoff, uint64_t* partial, uint32_t* big, uint32_t* nbig,
                   uint32_t* huge, uint32_t* nhuge, hipStream_t st) {
    // qcnt[nq] stays 0, so qoff[nq] = total rows
    const uint32_t n = nq + 1, tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(kTileSums, dim3(tiles), dim3(256), 0, st, qcnt, n, partial);
    hipLaunchKernelGGL(kScanPartials, dim3(1), dim3(256), 0, st, partial, tiles);
    hipLaunchKernelGGL(kScanTiles, dim3(tiles), dim3(256), 0, st, qcnt, n, partial, qoff, big, nbig, huge, nhuge);
    SH_HIP(hipGetLastError());
}

uint32_t scanTiles(uint32_t nq) { return (nq + 1 + kScanTile - 1) / kScanTile; }

__global__ void kBatchTotals(const uint32_t* __restrict__ small, const uint64_t* __restrict__ rowTotal,
                             const uint32_t* __restrict__ segCounts, uint32_t* __restrict__ out) {
    const uint32_t i = threadIdx.x;
    if (i < 8) out[i] = small[i];
    else if (i < 10) out[i] = (uint32_t)(*rowTotal >> (32 * (i - 8)));
    else if (i < 12) out[i] = segCounts[i - 10];
}

void launchBatchTotals(const uint32_t* small, const uint64_t* rowTotal, const uint32_t* segCounts, uint32_t* out,
                       hipStream_t st) {
    hipLaunchKernelGGL(kBatchTotals, dim3(1), dim3(64), 0, st, small, rowTotal, segCounts, out);
    SH_HIP(hipGetLastError());
}

void launchLocate(const LocateArgs& a, bool count, hipStream_t st) {
    if (a.nhits == 0) return;
    const uint64_t blocks = std::min<uint64_t>((a.nhits + 255) / 256, 65536);
    if (count) hipLaunchKernelGGL(kLocate<true>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    else       hipLaunchKernelGGL(kLocate<false>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    SH_HIP(hipGetLastError());
}

size_t bigSortTempBytes(uint64_t rows, uint32_t nbig) {
    size_t tb = 0;
    rocprim::transform_iterator<const uint32_t*, SegOff, uint32_t> bi(nullptr, SegOff{nullptr, 0});
    rocprim::transform_iterator<const uint32_t*, SegOff, uint32_t> ei(nullptr, SegOff{nullptr, 1});
    SH_HIP(rocprim::segmented_radix_sort_keys(nullptr, tb, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                              (unsigned)rows, nbig, bi, ei, 0, 36, (hipStream_t)0));
    return tb;
}

void sortDecode(uint64_t* k0, uint64_t* k1, uint64_t rows, const uint64_t* qoff, uint32_t nq, const uint32_t* big,
                uint32_t nbig, const uint32_t* huge, uint32_t nhuge, uint64_t qidBase, const uint64_t* starts,
                uint32_t nrec, sahara_hit* out, void* tmp, size_t tmpBytes, hipStream_t st) {
    if (rows == 0) return;
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((nq + 255) / 256, 65536));
    hipLaunchKernelGGL(kSortDecode, dim3(blocks), dim3(256), 0, st, k0, qoff, nq, qidBase, starts, nrec, out);
    SH_HIP(hipGetLastError());
    if (nbig) {  // long segments in LDS; huge ones skipped there
        hipLaunchKernelGGL(kSortBigLds, dim3(std::min<uint32_t>(nbig, 4096)), dim3(256), 0, st, k0, qoff, big, nbig,
                           qidBase, starts, nrec, out);
        SH_HIP(hipGetLastError());
    }
    if (nhuge == 0) return;
    rocprim::transform_iterator<const uint32_t*, SegOff, uint32_t> bi(huge, SegOff{qoff, 0});
    rocprim::transform_iterator<const uint32_t*, SegOff, uint32_t> ei(huge, SegOff{qoff, 1});
    size_t tb = tmpBytes;
    SH_HIP(rocprim::segmented_radix_sort_keys(tmp, tb, (const uint64_t*)k0, k1, (unsigned)rows, nhuge, bi, ei, 0, 36,
                                              st));
    hipLaunchKernelGGL(kDecodeBig, dim3(std::min<uint32_t>(nhuge, 65536)), dim3(256), 0, st, k1, qoff, huge, nhuge,
                       qidBase, starts, nrec, out);
    SH_HIP(hipGetLastError());
}

void launchPackPatterns3(const uint8_t* src, uint64_t npat, uint32_t m, uint32_t patBlocks, uint4* dst,
                         hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>((npat * patBlocks + 255) / 256, 65536);
    hipLaunchKernelGGL(kPackPatterns3, dim3((unsigned)blocks), dim3(256), 0, st, src, npat, m, patBlocks, dst);
    SH_HIP(hipGetLastError());
}

void launchDigest(const sahara_hit* h, uint64_t n, unsigned long long* out, hipStream_t st) {
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(kDigest, dim3((unsigned)blocks), dim3(256), 0, st, h, n, out);
    SH_HIP(hipGetLastError());
}

void launchCopyHits(const sahara_hit* h, uint64_t n, uint64_t qidOffset, sahara_hit* dst, hipStream_t st) {
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(kCopyHits, dim3((unsigned)blocks), dim3(256), 0, st, h, n, qidOffset, dst);
    SH_HIP(hipGetLastError());
}

}  // namespace sahara
