// search.hip — search-scheme DFS + locate on the GPU-resident FM-index (gfx950).
//
// Replaces fmc::search_ng24::search<Edit> (/root/reference/src/sahara/search.cpp:227,230)
// and fmc::LocateLinear (search.cpp:244-250) — semantics policy P0,
// docs/semantics.md; CPU restatement in oracle/oracle.cpp (Searcher::visit).
//
// Execution model (one lane = one DFS, the wave shares the work queue):
//   * Work items are (pattern, search) pairs. A lane with nothing to do takes
//     the next item; all idle lanes of a wave are served by ONE atomic on the
//     item counter (ballot + mbcnt prefix compaction).
//   * Each lane walks its search tree depth-first. The node being expanded
//     stays in registers; at every expansion the match child is pushed first
//     and all error children above it, and one error child continues in
//     registers. Hence the stack only holds siblings of error edges on the
//     current path: at most k * (2*sigma - 2) entries (k <= 15), independent
//     of the pattern length. Stacks live in HBM interleaved [depth][lane] so a
//     wave's pushes/pops at equal depth coalesce; the hot top sits in L2.
//   * An expansion ranks all sigma-1 symbols at lo and lo+len on the BWT of
//     the extension side: one 64-B Occ line per distinct 64-row block (1 or 2
//     lines), coalesced 16-B loads, popcount arithmetic — no LDS, no MFMA.
//   * Leaves (pos == len) are compacted to the hit buffer with a wave ballot
//     + one atomic per wave. Overflow of the hit buffer is flagged and the
//     host re-runs the batch with a larger buffer; nothing is truncated.
// Locate: one lane per reported cursor walks LF (<= rate-1 steps) on the
// forward lines to a sampled row; each step is one 64-B line. Records are
// packed into u64 keys (qid, text position, e) and radix-sorted for the
// canonical (qid, seq_id, pos, e) order.

#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#include "search.h"

namespace sahara {
namespace {

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
        r1 = *reinterpret_cast<const uint4*>(addrE + half);
        r2 = *reinterpret_cast<const uint4*>(addrE + 32 + half);
    }
    if (needO) {
        r3 = *reinterpret_cast<const uint4*>(addrO + half);
        r4 = *reinterpret_cast<const uint4*>(addrO + 32 + half);
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

constexpr uint32_t kWorkChunk = 256;  // items a wave takes per atomic
constexpr uint32_t kHitChunk = 64;    // hit slots a wave reserves per atomic
constexpr uint32_t kLdsDepth = 4;     // DFS stack levels kept in LDS (16 KB per block)

template <int SIGMA, bool EDIT, bool COUNT>
__global__ __launch_bounds__(256) void kSearch(SearchArgs a) {
    extern __shared__ uint32_t sch[];
    for (uint32_t i = threadIdx.x; i < a.nsearch * a.m; i += blockDim.x) sch[i] = a.scheme[i];
    __syncthreads();

    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t ltMask = (1ull << lane) - 1ull;
    const bool odd = lane & 1u;
    // DFS stack: the bottom kLdsDepth levels live in LDS ([level][thread],
    // conflict-free 16-B rows when lanes sit at equal depth), deeper levels
    // spill to HBM ([level][grid thread]). Typical depth stays in LDS.
    __shared__ uint4 lstk[kLdsDepth][256];
    uint4* stk = a.stack + gtid;
    auto spush = [&](uint32_t d, const uint4& v) {
        if (d < kLdsDepth) lstk[d][threadIdx.x] = v;
        else stk[(size_t)(d - kLdsDepth) * T] = v;
    };
    auto spop = [&](uint32_t d) -> uint4 {
        return d < kLdsDepth ? lstk[d][threadIdx.x] : stk[(size_t)(d - kLdsDepth) * T];
    };

    uint32_t sp = 0, pid = 0, sOff = 0;
    bool have = false, exhausted = false;
    uint32_t qNext = 0, qEnd = 0, hNext = 0, hEnd = 0, filled = 0;  // wave-uniform
    bool qDone = false;
    uint4 cur = make_uint4(0, 0, 0, 0);
    uint64_t cNodes = 0, cRank = 0, cLines = 0, cText = 0, cConv = 0;

    for (;;) {
        // ---- refill idle lanes from the wave's private item range; the wave
        // takes kWorkChunk items per atomic on the global counter, so one
        // counter word serves the whole grid without saturating
        const bool need = !have && sp == 0 && !exhausted;
        uint64_t pending = __ballot(need);
        while (pending) {  // wave-uniform
            if (qNext >= qEnd) {
                if (qDone) break;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(a.work, kWorkChunk);
                base = __shfl(base, 0);
                if (base >= a.nitems) { qDone = true; break; }
                qNext = base;
                qEnd = min(base + kWorkChunk, a.nitems);
            }
            const uint32_t take = min(qEnd - qNext, (uint32_t)__popcll(pending));
            const uint32_t rank = (uint32_t)__popcll(pending & ltMask);
            const bool mine = ((pending >> lane) & 1ull) && rank < take;
            if (mine) {
                const uint32_t item = qNext + rank;
                pid = item / a.nsearch;
                sOff = (item - pid * a.nsearch) * a.m;
                cur = make_uint4(0u, 0u, a.n, kDeltaZero);
                have = true;
            }
            pending &= ~__ballot(mine);
            qNext += take;
        }
        if (qDone && need && !have) exhausted = true;
        if (!have && sp > 0) {
            --sp;
            cur = spop(sp);
            have = true;
        }
        if (!__any(have)) break;

        // ---- leaves -> hit buffer: ballot + prefix compaction into the wave's
        // reserved slot range; a new range of kHitChunk slots costs one atomic
        const uint32_t pos = cur.w & 0xFFFFu;
        const bool leaf = have && pos == a.m;
        const uint64_t lm = __ballot(leaf);
        if (lm) {
            const uint32_t cnt = (uint32_t)__popcll(lm);
            const uint32_t rank = (uint32_t)__popcll(lm & ltMask);
            const uint32_t avail = hEnd - hNext;
            uint32_t base = 0;
            if (cnt > avail) {
                if (lane == 0) base = atomicAdd(a.hitCount, kHitChunk);
                base = __shfl(base, 0);
            }
            if (leaf) {
                const uint32_t idx = rank < avail ? hNext + rank : base + (rank - avail);
                const bool known = (cur.w & kTextBit) != 0;
                if (idx < a.hitCap)
                    a.hits[idx] = make_uint4(pid, cur.x, known ? 1u : cur.z, ((cur.w >> 16) & 0xFu) | (known ? kPosKnown : 0u));
                else atomicOr(a.flags, 2u);
                have = false;
            }
            if (cnt > avail) { hNext = base + (cnt - avail); hEnd = base + kHitChunk; }
            else hNext += cnt;
            filled += cnt;
        }
        // ---- decode the node (per lane)
        uint32_t e = 0, lastL = 0, lastR = 0, cq = 0, lb = 0, ub = 0;
        bool right = false, matchOK = false, misOK = false, delOK = false, insOK = false, text = false;
        uint32_t lo = 0, hi = 0, tc = 0;
        bool needA = false, needB = false;
        if (have) {
            e = (cur.w >> 16) & 0xFu;
            lastL = (cur.w >> 20) & 3u;
            lastR = (cur.w >> 22) & 3u;
            const uint32_t se = sch[sOff + pos];
            const uint32_t q = se & 0xFFFFu;
            lb = (se >> 16) & 0xFu;
            ub = (se >> 20) & 0xFu;
            right = (se >> 24) & 1u;
            cq = a.pats[(size_t)pid * a.m + q];
            const uint32_t side = right ? lastR : lastL;
            matchOK = lb <= e && e <= ub;
            misOK = lb <= e + 1 && e + 1 <= ub;
            delOK = EDIT && pos > 0 && e + 1 <= ub && side != OP_I;
            insOK = EDIT && misOK && side != OP_D;
            text = (cur.w & kTextBit) != 0;
            if (!text && a.verify && cur.z == 1u) {
                // singleton interval: resolve its text position once (full SA)
                // and continue the same DFS against the resident text
                const uint32_t p = a.sa[cur.x];
                const uint32_t tlen = pos + metaDelta(cur.w) - 16u;
                cur = make_uint4(p, p + tlen, 1u, cur.w | kTextBit);
                text = true;
                if (COUNT) ++cConv;
            }
            if (text) {
                const uint32_t tp = right ? cur.y : cur.x - 1u;  // next text symbol
                const bool inside = right ? (cur.y < a.n) : (cur.x > 0u);
                if (inside && (matchOK || misOK || delOK)) tc = (a.text4[tp >> 1] >> ((tp & 1u) * 4u)) & 0xFu;
            } else {
                lo = right ? cur.y : cur.x;
                hi = lo + cur.z;
                needA = matchOK || misOK || delOK;
                needB = needA && (hi >> 6) != (lo >> 6);
            }
        }

        // ---- pair-cooperative Occ line fetch (wave-uniform). Lanes 2i, 2i+1
        // fetch each other's lines together: every load instruction touches
        // at most 32 distinct 64-B lines (two lanes per line), which keeps
        // address translation off the critical path on a multi-GB index
        // (tools/gather_bench: 49.8 vs 21.7 Glines/s at 7 GB).
        const uint64_t ownA = (uint64_t)(right ? a.occR : a.occF) + (uint64_t)(lo >> 6) * 64u;
        const uint64_t ownB = (uint64_t)(right ? a.occR : a.occF) + (uint64_t)(hi >> 6) * 64u;
        uint32_t ca[5], cb[5];
        uint64_t pa[3], pb[3];
        fetchLinePair(ownA, needA, odd, ca, pa);
        fetchLinePair(ownB, needB, odd, cb, pb);

        if (have) {
        // ---- expand one node
        const uint32_t dl = metaDelta(cur.w);
        auto meta = [&](uint32_t npos, uint32_t ne, uint32_t op) -> uint32_t {
            const uint32_t nl = pos == 0 ? op : (right ? lastL : op);
            const uint32_t nr = pos == 0 ? op : (right ? op : lastR);
            const uint32_t nd = dl + (op == OP_D ? 1u : 0u) - (op == OP_I ? 1u : 0u);
            return npos | (ne << 16) | (nl << 20) | (nr << 22) | (cur.w & kTextBit) | (nd << 25);
        };
        if (COUNT) ++cNodes;

        // child c = (fx[c], fy[c], occ[c]): forward / reverse lower bounds of an
        // FM child, or the [start, end) text span of a text child
        uint32_t occ[SIGMA], fx[SIGMA], fy[SIGMA];
#pragma unroll
        for (int c = 0; c < SIGMA; ++c) occ[c] = fx[c] = fy[c] = 0;
        if (text) {
            // the only symbol that can extend a singleton is the text's own
            if (COUNT) ++cText;
            const uint32_t ns = right ? cur.x : cur.x - 1u, ne = right ? cur.y + 1u : cur.y;
#pragma unroll
            for (int c = 1; c < SIGMA; ++c) {  // branch-free: keeps the arrays in registers
                occ[c] = (uint32_t)c == tc ? 1u : 0u;
                fx[c] = ns;
                fy[c] = ne;
            }
        } else if (needA) {
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
            // bidirectional update: the other side moves by the occurrences of
            // the smaller symbols, '$' first
            uint32_t acc = (right ? cur.x : cur.y) + (cur.z - sum);
#pragma unroll
            for (int c = 1; c < SIGMA; ++c) {
                fx[c] = right ? acc : base[c];
                fy[c] = right ? base[c] : acc;
                acc += occ[c];
            }
        }
        auto child = [&](int c, uint32_t m) -> uint4 {
            return make_uint4(fx[c], fy[c], occ[c], m);
        };
        // count error children; find the match child
        uint32_t nErr = insOK ? 1u : 0u;
        bool hasM = false;
        uint4 mChild = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int c = 1; c < SIGMA; ++c) {
            if (occ[c]) {
                if ((uint32_t)c == cq) {
                    hasM = matchOK;
                    mChild = child(c, meta(pos + 1, e, OP_MS));
                } else {
                    nErr += misOK ? 1u : 0u;
                }
                nErr += delOK ? 1u : 0u;
            }
        }
        bool kept = false;
        uint4 next = make_uint4(0, 0, 0, 0);
        auto push = [&](const uint4& v) {
            if (sp < a.stackCap) {
                spush(sp, v);
                ++sp;
            } else {
                atomicOr(a.flags, 1u);
            }
        };
        auto emit = [&](const uint4& v) {
            if (!kept) { next = v; kept = true; }
            else push(v);
        };
        if (hasM && nErr) push(mChild);  // match child below all its error siblings
        if (insOK) emit(make_uint4(cur.x, cur.y, cur.z, meta(pos + 1, e + 1, OP_I)));
#pragma unroll
        for (int c = 1; c < SIGMA; ++c) {
            if (occ[c]) {
                if ((uint32_t)c != cq && misOK) emit(child(c, meta(pos + 1, e + 1, OP_MS)));
                if (delOK) emit(child(c, meta(pos, e + 1, OP_D)));
            }
        }
        if (!kept && hasM) { next = mChild; kept = true; }
        have = kept;
        cur = next;
        }  // have
    }
    // unused tail of the wave's last slot range: empty cursors (len 0)
    for (uint32_t i = hNext + lane; i < hEnd; i += 64)
        if (i < a.hitCap) a.hits[i] = make_uint4(0u, 0u, 0u, 0u);
    if (lane == 0 && filled) atomicAdd(a.filled, filled);
    if (COUNT) {
        atomicAdd(a.counters + 0, (unsigned long long)cNodes);
        atomicAdd(a.counters + 1, (unsigned long long)cRank);
        atomicAdd(a.counters + 2, (unsigned long long)cLines);
        atomicAdd(a.counters + 5, (unsigned long long)cText);
        atomicAdd(a.counters + 6, (unsigned long long)cConv);
    }
}

// One lane per reported cursor: locate every row of [lb, lb+len).
template <bool COUNT>
__global__ __launch_bounds__(256) void kLocate(LocateArgs a) {
    uint64_t steps = 0;
    for (uint64_t h = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; h < a.nhits;
         h += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 hit = a.hits[h];
        const uint64_t out = a.rowOff[h];
        const uint64_t e = hit.w & 0xFu;
        if (hit.w & kPosKnown) {  // resolved during the search (text mode)
            a.keys[out] = ((uint64_t)hit.x << 36) | ((uint64_t)hit.y << 4) | e;
            continue;
        }
        if (a.useSA) {  // full SA resident: one read per row
            for (uint32_t j = 0; j < hit.z; ++j)
                a.keys[out + j] = ((uint64_t)hit.x << 36) | ((uint64_t)a.sa[hit.y + j] << 4) | e;
            continue;
        }
        for (uint32_t j = 0; j < hit.z; ++j) {
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
            a.keys[out + j] = ((uint64_t)hit.x << 36) | (gpos << 4) | e;
        }
    }
    if (COUNT && steps) atomicAdd(a.counters, (unsigned long long)steps);
}

__global__ void kDecode(const uint64_t* __restrict__ keys, uint64_t n, uint64_t qidBase,
                        const uint64_t* __restrict__ starts, uint32_t nrec, sahara_hit* __restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const uint64_t gpos = (k >> 4) & 0xFFFFFFFFull;
        uint32_t lo = 0, hi = nrec;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (starts[mid] <= gpos) lo = mid; else hi = mid;
        }
        sahara_hit h;
        h.qid = qidBase + (k >> 36);
        h.seq_id = lo;
        h.err = (uint32_t)(k & 15u);
        h.pos = gpos - starts[lo];
        out[i] = h;
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

struct HitLen {
    __host__ __device__ uint64_t operator()(const uint4& h) const { return (uint64_t)h.z; }
};

template <int SIGMA>
void launchSearchT(const SearchArgs& a, bool edit, bool count, dim3 grid, size_t lds, hipStream_t st) {
    if (edit) {
        if (count) hipLaunchKernelGGL((kSearch<SIGMA, true, true>), grid, dim3(256), lds, st, a);
        else       hipLaunchKernelGGL((kSearch<SIGMA, true, false>), grid, dim3(256), lds, st, a);
    } else {
        if (count) hipLaunchKernelGGL((kSearch<SIGMA, false, true>), grid, dim3(256), lds, st, a);
        else       hipLaunchKernelGGL((kSearch<SIGMA, false, false>), grid, dim3(256), lds, st, a);
    }
}

}  // namespace

int searchBlocksPerCU(uint32_t sigma, bool edit, size_t lds) {
    int b = 0;
    const void* f;
    if (sigma == 5) f = edit ? (const void*)kSearch<5, true, false> : (const void*)kSearch<5, false, false>;
    else            f = edit ? (const void*)kSearch<6, true, false> : (const void*)kSearch<6, false, false>;
    SH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, 256, lds));
    return b < 1 ? 1 : b;
}

void launchSearch(const SearchArgs& a, uint32_t sigma, bool edit, bool count, uint32_t blocks, size_t lds,
                  hipStream_t st) {
    if (sigma == 5) launchSearchT<5>(a, edit, count, dim3(blocks), lds, st);
    else            launchSearchT<6>(a, edit, count, dim3(blocks), lds, st);
    SH_HIP(hipGetLastError());
}

size_t rowOffsetsTempBytes(uint64_t nhits) {
    size_t tb = 0;
    rocprim::transform_iterator<const uint4*, HitLen, uint64_t> it(nullptr, HitLen());
    SH_HIP(rocprim::exclusive_scan(nullptr, tb, it, (uint64_t*)nullptr, (uint64_t)0, (size_t)nhits + 1,
                                   rocprim::plus<uint64_t>(), (hipStream_t)0));
    return tb;
}

void rowOffsets(const uint4* hits, uint64_t nhits, uint64_t* off, void* tmp, size_t tmpBytes, hipStream_t st) {
    // off[nhits] = total rows (hits[nhits] must be readable: caller zeroes it)
    rocprim::transform_iterator<const uint4*, HitLen, uint64_t> it(hits, HitLen());
    size_t tb = tmpBytes;
    SH_HIP(rocprim::exclusive_scan(tmp, tb, it, off, (uint64_t)0, (size_t)nhits + 1, rocprim::plus<uint64_t>(),
                                   st));
}

void launchLocate(const LocateArgs& a, bool count, hipStream_t st) {
    if (a.nhits == 0) return;
    const uint64_t blocks = std::min<uint64_t>((a.nhits + 255) / 256, 65536);
    if (count) hipLaunchKernelGGL(kLocate<true>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    else       hipLaunchKernelGGL(kLocate<false>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    SH_HIP(hipGetLastError());
}

size_t sortTempBytes(uint64_t n) {
    size_t tb = 0;
    rocprim::double_buffer<uint64_t> kb(nullptr, nullptr);
    SH_HIP(rocprim::radix_sort_keys(nullptr, tb, kb, (size_t)n, 0, 64, (hipStream_t)0));
    return tb;
}

uint64_t* sortKeys(uint64_t* k0, uint64_t* k1, uint64_t n, unsigned endBit, void* tmp, size_t tmpBytes,
                   hipStream_t st) {
    if (n == 0) return k0;
    rocprim::double_buffer<uint64_t> kb(k0, k1);
    size_t tb = tmpBytes;
    SH_HIP(rocprim::radix_sort_keys(tmp, tb, kb, (size_t)n, 0, endBit, st));
    return kb.current();
}

void launchDecode(const uint64_t* keys, uint64_t n, uint64_t qidBase, const uint64_t* starts, uint32_t nrec,
                  sahara_hit* out, hipStream_t st) {
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(kDecode, dim3((unsigned)blocks), dim3(256), 0, st, keys, n, qidBase, starts, nrec, out);
    SH_HIP(hipGetLastError());
}

void launchDigest(const sahara_hit* h, uint64_t n, unsigned long long* out, hipStream_t st) {
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(kDigest, dim3((unsigned)blocks), dim3(256), 0, st, h, n, out);
    SH_HIP(hipGetLastError());
}

}  // namespace sahara
