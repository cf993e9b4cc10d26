// index_build.hip — GPU construction of the bidirectional FM-index (gfx950).
//
// Restates `sahara index` (/root/reference/src/sahara/index.cpp:41-112): the
// records are concatenated with one '$' (rank 0) after each, a suffix array
// is built for the text and for the per-record reversed text, and from it the
// two BWTs, the C array and the SA samples (samplingRate 16, index.cpp:87).
// Upstream does this on one CPU thread with libsais (fmindex-collection
// v1.1.0, absent here); this build uses GPU prefix doubling instead:
//   round 0: sort suffixes by their first 21 symbols packed 3 bits each,
//   round r: sort by (rank of the 2^r*21-prefix at i, rank at i + 2^r*21),
// with rocPRIM's onesweep radix sort (u64 keys, u32 suffix ids), until every
// rank group is a singleton. Random text finishes after 2 sorts at 3 Gbp.
// Sampling: row i is sampled iff the position of
// SA[i] inside its record is a multiple of the rate or is the record's
// delimiter. Record starts and delimiters are therefore sampled and no LF
// walk (locate, densification) ever steps through a '$' — where LF is not
// order-preserving for a text with several delimiters.

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <rocprim/rocprim.hpp>

#include "device_index.h"

namespace sahara {
namespace {

constexpr int kTB = 256;

inline unsigned gridFor(uint64_t n, unsigned cap = 65535u * 4u) {
    uint64_t g = (n + kTB - 1) / kTB;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

__device__ inline uint32_t recordOf(const uint64_t* starts, uint32_t nrec, uint64_t p) {
    uint32_t lo = 0, hi = nrec;  // last start <= p
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= p) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void kInitKeys(const uint8_t* __restrict__ T, uint64_t N, uint64_t* __restrict__ keys,
                          uint32_t* __restrict__ vals) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = 0;
#pragma unroll
        for (int j = 0; j < 21; ++j) {
            const uint64_t p = i + j;
            const uint64_t c = p < N ? (uint64_t)T[p] + 1u : 0u;
            k = (k << 3) | c;
        }
        keys[i] = k;
        vals[i] = (uint32_t)i;
    }
}

// g[i] = i at the head of a group of equal keys, 0 otherwise; counts heads.
__global__ void kHeads(const uint64_t* __restrict__ keys, uint64_t N, uint32_t* __restrict__ g,
                       unsigned long long* __restrict__ nheads) {
    uint32_t local = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const bool head = (i == 0) || keys[i] != keys[i - 1];
        g[i] = head ? (uint32_t)i : 0u;
        local += head;
    }
    // wave reduction then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(nheads, (unsigned long long)local);
}

__global__ void kScatterRank(const uint32_t* __restrict__ vals, const uint32_t* __restrict__ g, uint64_t N,
                             uint32_t* __restrict__ isa) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x)
        isa[vals[i]] = g[i];
}

__global__ void kPairKeys(const uint32_t* __restrict__ isa, uint64_t N, uint64_t h, uint64_t* __restrict__ keys,
                          uint32_t* __restrict__ vals) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t hi = isa[i];
        const uint64_t lo = (i + h < N) ? (uint64_t)isa[i + h] + 1u : 0u;
        keys[i] = (hi << 32) | lo;
        vals[i] = (uint32_t)i;
    }
}

__global__ void kReverseRecords(const uint8_t* __restrict__ T, uint64_t N, const uint64_t* __restrict__ starts,
                                const uint64_t* __restrict__ lens, uint32_t nrec, uint8_t* __restrict__ R) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = recordOf(starts, nrec, i);
        const uint64_t off = i - starts[r];
        R[i] = off < lens[r] ? T[starts[r] + lens[r] - 1 - off] : (uint8_t)0;
    }
}

__global__ void kBwt(const uint8_t* __restrict__ T, const uint32_t* __restrict__ sa, uint64_t N,
                     uint8_t* __restrict__ bwt) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = sa[i];
        bwt[i] = T[p ? p - 1 : N - 1];
    }
}

// One thread per 64-row block: sampled-row word.
__global__ void kSampledBits(const uint32_t* __restrict__ sa, uint64_t N, const uint64_t* __restrict__ starts,
                             uint32_t nrec, uint32_t rate, uint64_t* __restrict__ bits) {
    const uint64_t nb = N / 64 + 1;
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb;
         b += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t w = 0;
        for (uint32_t j = 0; j < 64; ++j) {
            const uint64_t i = b * 64 + j;
            if (i >= N) break;
            const uint64_t p = sa[i];
            const uint32_t r = recordOf(starts, nrec, p);
            const uint64_t off = p - starts[r];
            const uint64_t len = (r + 1 < nrec ? starts[r + 1] : N) - starts[r] - 1;
            if (off % rate == 0 || off == len) w |= 1ull << j;  // delimiters always sampled
        }
        bits[b] = w;
    }
}

struct Cnt6 {
    uint32_t c[6];  // symbols 1..5, then sampled rows
};
struct Cnt6Plus {
    __host__ __device__ Cnt6 operator()(const Cnt6& a, const Cnt6& b) const {
        Cnt6 r;
#pragma unroll
        for (int i = 0; i < 6; ++i) r.c[i] = a.c[i] + b.c[i];
        return r;
    }
};

// One thread per 64-position block: local symbol counts + bit planes.
__global__ void kLinesLocal(const uint8_t* __restrict__ bwt, uint64_t N, const uint64_t* __restrict__ sampled,
                            OccLine* __restrict__ lines, Cnt6* __restrict__ counts) {
    const uint64_t nb = N / 64 + 1;
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb;
         b += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t p0 = 0, p1 = 0, p2 = 0;
        Cnt6 c = {{0, 0, 0, 0, 0, 0}};
        const uint64_t base = b * 64;
        if (base + 64 <= N) {
            const uint4* src = reinterpret_cast<const uint4*>(bwt + base);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint4 q = src[v];
                const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const uint32_t s = (w[t >> 2] >> ((t & 3) * 8)) & 0xffu;
                    const int j = v * 16 + t;
                    p0 |= (uint64_t)(s & 1u) << j;
                    p1 |= (uint64_t)((s >> 1) & 1u) << j;
                    p2 |= (uint64_t)((s >> 2) & 1u) << j;
                }
            }
        } else {
            for (uint64_t j = 0; j < 64 && base + j < N; ++j) {
                const uint32_t s = bwt[base + j];
                p0 |= (uint64_t)(s & 1u) << j;
                p1 |= (uint64_t)((s >> 1) & 1u) << j;
                p2 |= (uint64_t)((s >> 2) & 1u) << j;
            }
        }
        const uint64_t valid = (base + 64 <= N) ? ~0ull : lowMask((uint32_t)(N - base));
        const uint64_t pl[3] = {p0, p1, p2};
#pragma unroll
        for (uint32_t s = 1; s <= 5; ++s) c.c[s - 1] = (uint32_t)__popcll(symMask(pl, s) & valid);
        const uint64_t sw = sampled ? sampled[b] : 0ull;
        c.c[5] = (uint32_t)__popcll(sw);
        OccLine L;
        L.plane[0] = p0;
        L.plane[1] = p1;
        L.plane[2] = p2;
        L.sampled = sw;
        L.reserved = 0;
        lines[b] = L;  // counts filled after the scan
        counts[b] = c;
    }
}

__global__ void kLinesCounts(OccLine* __restrict__ lines, const Cnt6* __restrict__ scanned, uint64_t nb) {
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const Cnt6 c = scanned[b];
#pragma unroll
        for (int s = 0; s < 5; ++s) lines[b].cnt[s] = c.c[s];
        lines[b].srank = c.c[5];
    }
}

__global__ void kSamples(const uint32_t* __restrict__ sa, uint64_t N, const OccLine* __restrict__ lines,
                         uint32_t* __restrict__ samples) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const OccLine& L = lines[i >> 6];
        const uint32_t o = (uint32_t)(i & 63);
        if ((L.sampled >> o) & 1ull) samples[L.srank + __popcll(L.sampled & lowMask(o))] = sa[i];
    }
}

__global__ void kDecodeBwt(const OccLine* __restrict__ lines, uint64_t N, uint8_t* __restrict__ bwt) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x)
        bwt[i] = (uint8_t)symAt(lines[i >> 6].plane, (uint32_t)(i & 63));
}

__global__ void kSampledWords(const OccLine* __restrict__ lines, uint64_t nb, uint64_t* __restrict__ w) {
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb;
         b += (uint64_t)gridDim.x * blockDim.x)
        w[b] = lines[b].sampled;
}


// text bytes (one symbol per byte) -> 4-bit packed, two symbols per byte
// text (one symbol per byte) -> 3-bit-plane blocks of 32 symbols (device_index.h)
__global__ void kPackText(const uint8_t* __restrict__ T, uint64_t N, uint4* __restrict__ t3) {
    const uint64_t nb = (N + 31) / 32;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nb;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t p0 = 0, p1 = 0, p2 = 0;
        const uint64_t base = 32 * i;
        const uint32_t cnt = (uint32_t)(N - base < 32 ? N - base : 32);
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t c = T[base + j];
            p0 |= (c & 1u) << j;
            p1 |= ((c >> 1) & 1u) << j;
            p2 |= ((c >> 2) & 1u) << j;
        }
        t3[i] = make_uint4(p0, p1, p2, 0u);
    }
}

__device__ __forceinline__ uint32_t rankAll(const OccLine& L, uint32_t row, uint32_t c) {
    // occurrences of symbol c in BWT[0, row); '$' (c = 0) by complement
    const uint32_t o = row & 63u;
    const uint64_t m = lowMask(o);
    if (c != 0) return L.cnt[c - 1] + (uint32_t)__popcll(symMask(L.plane, c) & m);
    uint32_t others = 0;
#pragma unroll
    for (uint32_t s = 1; s <= 5; ++s) others += L.cnt[s - 1] + (uint32_t)__popcll(symMask(L.plane, s) & m);
    return row - others;
}

// Densify the sampled SA to the full SA and recover the text from the BWT:
// every sampled row seeds a backward LF walk that stops at the next sampled
// row or at a record start, writing SA[row] = pos and T[pos-1] = BWT[row] on
// the way ('$' entries of T stay 0). Each row is visited by exactly one walk.
// A wave takes 1024 consecutive rows (16 Occ lines), compacts their sampled
// rows (about 1 in rate) with their text positions into an LDS list, and its
// lanes then walk one chain each: every lane of the wave has a walk in flight.
// (A lane per row, r5, left ~4 of 64 lanes walking: 238 ms at 3 Gbp, 12.6 G
// LF steps/s against the ~50 G random lines/s the gather ceiling allows.)
constexpr uint32_t kDensifyRows = 1024;  // rows per wave
__global__ __launch_bounds__(256) void kDensify(const OccLine* __restrict__ occ, uint64_t N,
                                                const uint32_t* __restrict__ samples, const uint64_t* __restrict__ C,
                                                uint32_t rate, uint32_t* __restrict__ sa, uint8_t* __restrict__ T,
                                                unsigned int* __restrict__ err) {
    __shared__ uint2 list[4][kDensifyRows];  // (row, text position) of the wave's sampled rows
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t nblk = (N + kDensifyRows - 1) / kDensifyRows;
    for (uint64_t blk = (uint64_t)blockIdx.x * 4 + w; blk < nblk; blk += (uint64_t)gridDim.x * 4) {
        // lane l looks at rows [16 l, 16 l + 16) of the block: a quarter of one line
        const uint64_t r16 = blk * kDensifyRows + 16u * lane;
        uint32_t bits = 0, k0 = 0;
        if (r16 < N) {
            const OccLine& L = occ[r16 >> 6];
            const uint32_t o = (uint32_t)(r16 & 63u);
            bits = (uint32_t)(L.sampled >> o) & 0xFFFFu;
            if (r16 + 16 > N) bits &= (1u << (uint32_t)(N - r16)) - 1u;
            k0 = L.srank + (uint32_t)__popcll(L.sampled & lowMask(o));  // the first one's sample index
        }
        const uint32_t cnt = (uint32_t)__popc(bits);
        uint32_t incl = cnt;  // inclusive prefix over the wave's lanes
#pragma unroll
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        const uint32_t total = __shfl(incl, 63);
        for (uint32_t at = incl - cnt, k = k0; bits; bits &= bits - 1u, ++at, ++k)
            list[w][at] = make_uint2((uint32_t)(r16 + (uint32_t)__builtin_ctz(bits)), samples[k]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t j = lane; j < total; j += 64) {
            uint32_t row = list[w][j].x;
            uint64_t pos = list[w][j].y;
            sa[row] = (uint32_t)pos;
            for (uint32_t step = 0;; ++step) {
                if (step > rate) { atomicOr(err, 1u); break; }
                const OccLine& L = occ[row >> 6];
                const uint32_t c = symAt(L.plane, row & 63u);
                if (pos == 0 || c == 0) break;  // record start: the '$' before it is sampled
                T[pos - 1] = (uint8_t)c;
                row = (uint32_t)C[c] + rankAll(L, row, c);
                --pos;
                const OccLine& L2 = occ[row >> 6];
                if ((L2.sampled >> (row & 63u)) & 1ull) break;
                sa[row] = (uint32_t)pos;
            }
        }
        __builtin_amdgcn_wave_barrier();  // the list is reused for the next block
    }
}

// Builds the suffix array of the device text T[0, N) into `sa`.
void suffixArray(const uint8_t* dT, uint64_t N, uint32_t* dSA, hipStream_t st) {
    DevBuf<uint64_t> k0, k1;
    DevBuf<uint32_t> v1, g, isa;
    k0.reserve(N);
    k1.reserve(N);
    v1.reserve(N);
    g.reserve(N);
    isa.reserve(N);
    DevBuf<unsigned long long> cnt;
    cnt.reserve(1);
    DevBuf<char> tmp;
    const unsigned grid = gridFor(N);

    hipLaunchKernelGGL(kInitKeys, dim3(grid), dim3(kTB), 0, st, dT, N, k0.ptr, dSA);
    SH_HIP(hipGetLastError());
    rocprim::double_buffer<uint64_t> kb(k0.ptr, k1.ptr);
    rocprim::double_buffer<uint32_t> vb(dSA, v1.ptr);
    size_t tmpBytes = 0;
    SH_HIP(rocprim::radix_sort_pairs(nullptr, tmpBytes, kb, vb, (size_t)N, 0, 64, st));
    size_t scanBytes = 0;
    SH_HIP(rocprim::inclusive_scan(nullptr, scanBytes, g.ptr, g.ptr, (size_t)N, rocprim::maximum<uint32_t>(), st));
    tmp.reserve(std::max(tmpBytes, scanBytes) + 256);
    size_t tb = tmp.cap;
    SH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, kb, vb, (size_t)N, 0, 63, st));

    uint64_t h = 21;
    for (int round = 0;; ++round) {
        SH_HIP(hipMemsetAsync(cnt.ptr, 0, sizeof(unsigned long long), st));
        hipLaunchKernelGGL(kHeads, dim3(grid), dim3(kTB), 0, st, kb.current(), N, g.ptr, cnt.ptr);
        SH_HIP(hipGetLastError());
        unsigned long long heads = 0;
        SH_HIP(hipMemcpyAsync(&heads, cnt.ptr, sizeof(heads), hipMemcpyDeviceToHost, st));
        SH_HIP(hipStreamSynchronize(st));
        if (heads == N) break;
        if (round > 40) throw Error("suffix array construction did not converge");
        tb = tmp.cap;
        SH_HIP(rocprim::inclusive_scan(tmp.ptr, tb, g.ptr, g.ptr, (size_t)N, rocprim::maximum<uint32_t>(), st));
        hipLaunchKernelGGL(kScatterRank, dim3(grid), dim3(kTB), 0, st, vb.current(), g.ptr, N, isa.ptr);
        hipLaunchKernelGGL(kPairKeys, dim3(grid), dim3(kTB), 0, st, isa.ptr, N, h, kb.current(), vb.current());
        SH_HIP(hipGetLastError());
        tb = tmp.cap;
        SH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, kb, vb, (size_t)N, 0, 64, st));
        h *= 2;
    }
    if (vb.current() != dSA)
        SH_HIP(hipMemcpyAsync(dSA, vb.current(), N * 4, hipMemcpyDeviceToDevice, st));
    SH_HIP(hipStreamSynchronize(st));
}

// BWT bytes (+ optional sampled words) -> Occ lines with prefix counts.
void buildLines(const uint8_t* dBwt, uint64_t N, const uint64_t* dSampled, DevBuf<OccLine>& lines,
                uint64_t totals[6], hipStream_t st) {
    const uint64_t nb = N / 64 + 1;
    lines.reserve(nb);
    DevBuf<Cnt6> counts;
    counts.reserve(nb + 1);
    const unsigned grid = gridFor(nb);
    hipLaunchKernelGGL(kLinesLocal, dim3(grid), dim3(kTB), 0, st, dBwt, N, dSampled, lines.ptr, counts.ptr);
    SH_HIP(hipGetLastError());
    SH_HIP(hipMemsetAsync(counts.ptr + nb, 0, sizeof(Cnt6), st));
    size_t tb = 0;
    Cnt6 zero = {{0, 0, 0, 0, 0, 0}};
    SH_HIP(rocprim::exclusive_scan(nullptr, tb, counts.ptr, counts.ptr, zero, (size_t)nb + 1, Cnt6Plus(), st));
    DevBuf<char> tmp;
    tmp.reserve(tb + 256);
    tb = tmp.cap;
    SH_HIP(rocprim::exclusive_scan(tmp.ptr, tb, counts.ptr, counts.ptr, zero, (size_t)nb + 1, Cnt6Plus(), st));
    hipLaunchKernelGGL(kLinesCounts, dim3(grid), dim3(kTB), 0, st, lines.ptr, counts.ptr, nb);
    SH_HIP(hipGetLastError());
    Cnt6 tot;
    SH_HIP(hipMemcpyAsync(&tot, counts.ptr + nb, sizeof(Cnt6), hipMemcpyDeviceToHost, st));
    SH_HIP(hipStreamSynchronize(st));
    for (int i = 0; i < 6; ++i) totals[i] = tot.c[i];
}

void setCommon(DeviceIndex& I, uint32_t sigma, uint64_t n, const uint64_t* recLens, uint64_t nrec, uint32_t rate,
               hipStream_t st) {
    I.sigma = sigma;
    I.n = n;
    I.rate = rate;
    I.recLens.assign(recLens, recLens + nrec);
    I.recStarts.resize(nrec);
    uint64_t s = 0;
    for (uint64_t r = 0; r < nrec; ++r) { I.recStarts[r] = s; s += recLens[r] + 1; }
    I.dRecStarts.reserve(nrec);
    SH_HIP(hipMemcpyAsync(I.dRecStarts.ptr, I.recStarts.data(), nrec * 8, hipMemcpyHostToDevice, st));
}

void setC(DeviceIndex& I, const uint64_t totals[6], uint64_t nrec) {
    uint64_t cnt[8] = {0};
    cnt[0] = nrec;  // one '$' per record
    for (uint32_t c = 1; c < I.sigma; ++c) cnt[c] = totals[c - 1];
    I.C[0] = 0;
    for (uint32_t c = 1; c <= I.sigma; ++c) I.C[c] = I.C[c - 1] + cnt[c - 1];
}

}  // namespace

// ----------------------------------------------------------- k-mer table ----
struct Cvec {
    uint64_t v[8];
};

// Level j of the table from level j-1: each string w extends to the right by
// A, C, G, T (extendRight on the reverse BWT: one rank of all symbols at lbRev
// and lbRev + len; the forward lb moves by the occurrences of the smaller
// symbols, '$' first). Empty intervals stay empty. At the last level (sa set)
// a string that occurs once also gets its text position, SA[lb], in the
// entry's fourth word: kSeedItems hands such a seed to the text phase as a
// task that needs no SA read of its own.
__global__ void kKmerLevel(const OccLine* __restrict__ occR, Cvec C, uint32_t sigma, const uint4* __restrict__ prev,
                           uint64_t count, uint4* __restrict__ next, const uint32_t* __restrict__ sa) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 w = prev[i];
        uint4 out[4] = {};
        if (w.z) {
            const uint32_t lo = w.y, hi = w.y + w.z;
            const OccLine& A = occR[lo >> 6];
            const OccLine& B = occR[hi >> 6];
            const uint64_t ml = lowMask(lo & 63u), mh = lowMask(hi & 63u);
            uint32_t occ[6] = {}, base[6] = {}, sum = 0;
            for (uint32_t c = 1; c < sigma; ++c) {
                const uint32_t rl = A.cnt[c - 1] + (uint32_t)__popcll(symMask(A.plane, c) & ml);
                const uint32_t rh = B.cnt[c - 1] + (uint32_t)__popcll(symMask(B.plane, c) & mh);
                occ[c] = rh - rl;
                base[c] = (uint32_t)C.v[c] + rl;
                sum += occ[c];
            }
            uint32_t acc = w.x + (w.z - sum);
            uint32_t j = 0;
            for (uint32_t c = 1; c < sigma; ++c) {
                const bool acgt = !(sigma == 6 && c == 4);  // N is not in the table
                if (acgt)
                    out[j++] = occ[c] ? make_uint4(acc, base[c], occ[c], sa && occ[c] == 1u ? sa[acc] : 0u)
                                      : make_uint4(0u, 0u, 0u, 0u);
                acc += occ[c];
            }
        }
        for (int j = 0; j < 4; ++j) next[i * 4 + j] = out[j];
    }
}

std::vector<uint64_t> splitRecords(const uint64_t* recLens, uint64_t nrec) {
    uint64_t limit = 0xFFFFFFFDull;  // n < 2^32 - 2 symbols per part, delimiters included
    if (const char* e = std::getenv("SAHARA_PART_SYMBOLS")) limit = std::max<uint64_t>(2, std::min<uint64_t>(limit, std::atoll(e)));
    std::vector<uint64_t> first{0};
    uint64_t n = 0;
    for (uint64_t r = 0; r < nrec; ++r) {
        if (recLens[r] + 1 > 0xFFFFFFFDull)
            throw Error("record " + std::to_string(r) + " alone exceeds 2^32 - 2 symbols (32-bit rows per part)");
        if (n && n + recLens[r] + 1 > limit) {
            first.push_back(r);
            n = 0;
        }
        n += recLens[r] + 1;
    }
    first.push_back(nrec);
    return first;
}

void buildFromText(DeviceIndex& I, const uint8_t* hostRanks, const uint64_t* recLens, uint64_t nrec, uint32_t sigma,
                   uint32_t rate, hipStream_t st, bool withKmer) {
    if (sigma != 5 && sigma != 6) throw Error("sigma must be 5 (dna4) or 6 (dna5)");
    if (nrec == 0) throw Error("reference is empty");
    if (rate == 0) throw Error("sampling rate must be > 0");
    uint64_t N = 0;
    for (uint64_t r = 0; r < nrec; ++r) N += recLens[r] + 1;
    if (N >= 0xFFFFFFFEull) throw Error("text too long for 32-bit rows (n must be < 2^32 - 2)");
    for (uint64_t i = 0, tot = N - nrec; i < tot; ++i)
        if (hostRanks[i] == 0 || hostRanks[i] >= sigma) throw Error("reference rank out of range");
    setCommon(I, sigma, N, recLens, nrec, rate, st);

    // text with delimiters, on device
    DevBuf<uint8_t> T, R, bwt;
    DevBuf<uint64_t> dLens;
    T.reserve(N + 16);
    R.reserve(N + 16);
    dLens.reserve(nrec);
    SH_HIP(hipMemcpyAsync(dLens.ptr, recLens, nrec * 8, hipMemcpyHostToDevice, st));
    SH_HIP(hipMemsetAsync(T.ptr, 0, N + 16, st));
    for (uint64_t r = 0, off = 0; r < nrec; ++r) {
        SH_HIP(hipMemcpyAsync(T.ptr + I.recStarts[r], hostRanks + off, recLens[r], hipMemcpyHostToDevice, st));
        off += recLens[r];
    }
    const unsigned grid = gridFor(N);
    hipLaunchKernelGGL(kReverseRecords, dim3(grid), dim3(kTB), 0, st, T.ptr, N, I.dRecStarts.ptr, dLens.ptr,
                       (uint32_t)nrec, R.ptr);
    SH_HIP(hipGetLastError());

    DevBuf<uint32_t> sa;
    sa.reserve(N);
    DevBuf<uint64_t> sampled;
    const uint64_t nb = N / 64 + 1;
    sampled.reserve(nb);
    bwt.reserve(N + 64);
    uint64_t totals[6];

    // forward direction: SA, BWT, sampling, lines, samples
    suffixArray(T.ptr, N, sa.ptr, st);
    hipLaunchKernelGGL(kBwt, dim3(grid), dim3(kTB), 0, st, T.ptr, sa.ptr, N, bwt.ptr);
    hipLaunchKernelGGL(kSampledBits, dim3(gridFor(nb)), dim3(kTB), 0, st, sa.ptr, N, I.dRecStarts.ptr,
                       (uint32_t)nrec, rate, sampled.ptr);
    SH_HIP(hipGetLastError());
    buildLines(bwt.ptr, N, sampled.ptr, I.occF, totals, st);
    setC(I, totals, nrec);
    I.nsamples = totals[5];
    I.samples.reserve(std::max<uint64_t>(I.nsamples, 1));
    hipLaunchKernelGGL(kSamples, dim3(grid), dim3(kTB), 0, st, sa.ptr, N, I.occF.ptr, I.samples.ptr);
    SH_HIP(hipGetLastError());
    // resident full SA + packed text for the search (locate = one read)
    I.saFull.reserve(N);
    SH_HIP(hipMemcpyAsync(I.saFull.ptr, sa.ptr, N * 4, hipMemcpyDeviceToDevice, st));
    I.text3.reserve(text3Blocks(N));
    SH_HIP(hipMemsetAsync(I.text3.ptr, 0, text3Blocks(N) * sizeof(uint4), st));
    hipLaunchKernelGGL(kPackText, dim3(gridFor((N + 31) / 32)), dim3(kTB), 0, st, T.ptr, N, I.text3.ptr);
    SH_HIP(hipGetLastError());

    // reverse direction: SA, BWT, lines (no sampling)
    suffixArray(R.ptr, N, sa.ptr, st);
    hipLaunchKernelGGL(kBwt, dim3(grid), dim3(kTB), 0, st, R.ptr, sa.ptr, N, bwt.ptr);
    SH_HIP(hipGetLastError());
    uint64_t totalsR[6];
    buildLines(bwt.ptr, N, nullptr, I.occR, totalsR, st);
    for (int c = 0; c < 5; ++c)
        if (totalsR[c] != totals[c]) throw Error("forward/reverse symbol counts differ");
    SH_HIP(hipStreamSynchronize(st));
    if (withKmer) buildKmerTable(I, kmerDepth(N), st);
}

void buildFromParts(DeviceIndex& I, uint32_t sigma, uint64_t n, const uint64_t* recLens, uint64_t nrec, uint32_t rate,
                    const uint8_t* bwtF, const uint8_t* bwtR, const uint64_t* sampledBits, const uint32_t* samples,
                    uint64_t nsamples, hipStream_t st, bool withKmer, const HostUpload* up) {
    auto upload = [up](void* dst, const void* src, size_t bytes, hipStream_t s) {
        if (up) (*up)(dst, src, bytes, s);
        else SH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    };
    if (sigma != 5 && sigma != 6) throw Error("sigma must be 5 (dna4) or 6 (dna5)");
    if (n >= 0xFFFFFFFEull) throw Error("text too long for 32-bit rows");
    setCommon(I, sigma, n, recLens, nrec, rate, st);
    // SAHARA_TIMING: where the load's time goes (stderr), from events between
    // its steps and the host clock
    struct Phases {
        bool on = std::getenv("SAHARA_TIMING") != nullptr;
        hipStream_t st;
        std::vector<std::pair<const char*, hipEvent_t>> ev;
        std::vector<double> host;
        std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
        void operator()(const char* what) {
            if (!on) return;
            hipEvent_t e;
            SH_HIP(hipEventCreate(&e));
            SH_HIP(hipEventRecord(e, st));
            ev.emplace_back(what, e);
            host.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        void report() {
            if (!on || ev.empty()) return;
            SH_HIP(hipEventSynchronize(ev.back().second));
            std::fprintf(stderr, "[sahara] index load (ms, device | host issue):");
            for (size_t i = 1; i < ev.size(); ++i) {
                float ms = 0;
                SH_HIP(hipEventElapsedTime(&ms, ev[i - 1].second, ev[i].second));
                std::fprintf(stderr, " %s %.1f | %.1f", ev[i].first, ms, host[i] - host[i - 1]);
            }
            std::fprintf(stderr, "\n");
        }
        ~Phases() {
            for (auto& x : ev) (void)hipEventDestroy(x.second);
        }
    } phase{};
    phase.st = st;
    phase("start");
    const uint64_t nb = n / 64 + 1;
    DevBuf<uint8_t> bwt, bwtRev;
    DevBuf<uint64_t> sampled;
    bwt.reserve(n + 64);
    sampled.reserve(nb);
    uint64_t totals[6], totalsR[6];
    upload(sampled.ptr, sampledBits, nb * 8, st);
    upload(bwt.ptr, bwtF, n, st);
    phase("bwtF up");
    buildLines(bwt.ptr, n, sampled.ptr, I.occF, totals, st);
    phase("occF");
    if (totals[5] != nsamples) throw Error("sampled bitvector and sample count disagree");
    setC(I, totals, nrec);
    I.nsamples = nsamples;
    I.samples.reserve(std::max<uint64_t>(nsamples, 1));
    upload(I.samples.ptr, samples, nsamples * 4, st);
    phase("samples up");
    // full SA + text from the sampled SA by bounded LF walks (the forward
    // BWT's buffer becomes the unpacked text); the reverse BWT goes up on a
    // second stream meanwhile (a pageable copy holds the host thread, not the
    // device), so its upload hides behind the walks
    I.saFull.reserve(n);
    DevBuf<uint64_t> dC;
    dC.reserve(8);
    SH_HIP(hipMemcpyAsync(dC.ptr, I.C, 8 * 8, hipMemcpyHostToDevice, st));
    DevBuf<unsigned int> err;
    err.reserve(1);
    SH_HIP(hipMemsetAsync(err.ptr, 0, 4, st));
    SH_HIP(hipMemsetAsync(bwt.ptr, 0, n + 64, st));
    hipLaunchKernelGGL(kDensify, dim3(gridFor((n + kDensifyRows - 1) / kDensifyRows * 64)), dim3(kTB), 0, st,
                       I.occF.ptr, n, I.samples.ptr, dC.ptr, rate, I.saFull.ptr, bwt.ptr, err.ptr);
    SH_HIP(hipGetLastError());
    phase("densify");
    I.text3.reserve(text3Blocks(n));
    SH_HIP(hipMemsetAsync(I.text3.ptr, 0, text3Blocks(n) * sizeof(uint4), st));
    hipLaunchKernelGGL(kPackText, dim3(gridFor((n + 31) / 32)), dim3(kTB), 0, st, bwt.ptr, n, I.text3.ptr);
    SH_HIP(hipGetLastError());
    phase("text");
    {
        struct Side {  // the reverse BWT's upload stream and the event st waits on
            hipStream_t s = nullptr;
            hipEvent_t e = nullptr;
            ~Side() {
                if (e) (void)hipEventDestroy(e);
                if (s) (void)hipStreamDestroy(s);
            }
        } side;
        SH_HIP(hipStreamCreateWithFlags(&side.s, hipStreamNonBlocking));
        SH_HIP(hipEventCreateWithFlags(&side.e, hipEventDisableTiming));
        bwtRev.reserve(n + 64);
        upload(bwtRev.ptr, bwtR, n, side.s);
        SH_HIP(hipEventRecord(side.e, side.s));
        SH_HIP(hipStreamWaitEvent(st, side.e, 0));
        phase("bwtR up (beside the walks)");
        buildLines(bwtRev.ptr, n, nullptr, I.occR, totalsR, st);
        phase("occR");
    }
    for (int c = 0; c < 5; ++c)
        if (totalsR[c] != totals[c]) throw Error("forward/reverse BWT symbol counts differ");
    unsigned int herr = 0;
    SH_HIP(hipMemcpyAsync(&herr, err.ptr, 4, hipMemcpyDeviceToHost, st));
    SH_HIP(hipStreamSynchronize(st));
    if (herr) throw Error("SA densification walk exceeded its bound (inconsistent .idx samples)");
    bwtRev.release();
    bwt.release();
    if (withKmer) buildKmerTable(I, kmerDepth(n), st);
    phase("kmer");
    phase.report();
}

uint32_t kmerDepth(uint64_t n, uint32_t tables) {
    uint32_t lg = 0;
    while (lg < 31 && (1ull << (2 * (lg + 1))) <= n) ++lg;  // floor(log4 n)
    int k = (int)lg + 1;
    if (const char* e = std::getenv("SAHARA_KMER")) k = std::atoi(e);
    k = std::max(0, std::min(k, 16));
    // the tables (16 B x 4^K each) and the build levels of one (2 x 16 B x
    // 4^(K-1)) take at most half of the free HBM, or, for the parts of a
    // multi-part index (built after all parts), three quarters of it less 16 GB
    // for the search's buffers (6 Gbp in two parts: two depth-16 tables, 137 GB)
    size_t freeB = 0, totalB = 0;
    const uint64_t budget = [&]() -> uint64_t {
        if (hipMemGetInfo(&freeB, &totalB) != hipSuccess) return UINT64_MAX;
        if (tables <= 1) return freeB / 2;
        const uint64_t q = (uint64_t)freeB / 4 * 3;
        return q > (16ull << 30) ? q - (16ull << 30) : 0;
    }();
    while (k > 0 && tables * (16ull << (2 * k)) + (32ull << (2 * (k - 1))) > budget) --k;
    return (uint32_t)k;
}

void buildKmerTable(DeviceIndex& I, uint32_t K, hipStream_t st) {
    I.kmerK = 0;
    I.kmer.release();
    if (K == 0) return;
    Cvec C;
    for (int c = 0; c < 8; ++c) C.v[c] = I.C[c];
    DevBuf<uint4> t0, t1;  // levels 0 .. K-1, alternating
    const uint64_t maxPrev = 1ull << (2 * (K - 1));
    t0.reserve(maxPrev);
    if (K > 1) t1.reserve(maxPrev);
    I.kmer.reserve(1ull << (2 * K));
    const uint4 root = make_uint4(0u, 0u, (uint32_t)I.n, 0u);
    SH_HIP(hipMemcpyAsync(t0.ptr, &root, sizeof(root), hipMemcpyHostToDevice, st));
    uint4* prev = t0.ptr;
    uint64_t count = 1;
    for (uint32_t j = 1; j <= K; ++j) {
        uint4* next = j == K ? I.kmer.ptr : (prev == t0.ptr ? t1.ptr : t0.ptr);
        hipLaunchKernelGGL(kKmerLevel, dim3((unsigned)std::min<uint64_t>((count + 255) / 256, 1u << 16)), dim3(256), 0,
                           st, I.occR.ptr, C, I.sigma, prev, count, next,
                           j == K && I.saFull.cap >= I.n ? I.saFull.ptr : nullptr);
        SH_HIP(hipGetLastError());
        count *= 4;
        prev = next;
    }
    SH_HIP(hipStreamSynchronize(st));
    I.kmerK = K;
    I.kmerPos = I.saFull.cap >= I.n;
}

void exportParts(const DeviceIndex& I, uint8_t* bwtF, uint8_t* bwtR, uint64_t* sampledBits, uint32_t* samples,
                 hipStream_t st) {
    const uint64_t N = I.n, nb = N / 64 + 1;
    DevBuf<uint8_t> bwt;
    bwt.reserve(N + 64);
    const unsigned grid = gridFor(N);
    if (bwtF) {
        hipLaunchKernelGGL(kDecodeBwt, dim3(grid), dim3(kTB), 0, st, I.occF.ptr, N, bwt.ptr);
        SH_HIP(hipMemcpyAsync(bwtF, bwt.ptr, N, hipMemcpyDeviceToHost, st));
        SH_HIP(hipStreamSynchronize(st));
    }
    if (bwtR) {
        hipLaunchKernelGGL(kDecodeBwt, dim3(grid), dim3(kTB), 0, st, I.occR.ptr, N, bwt.ptr);
        SH_HIP(hipMemcpyAsync(bwtR, bwt.ptr, N, hipMemcpyDeviceToHost, st));
        SH_HIP(hipStreamSynchronize(st));
    }
    if (sampledBits) {
        DevBuf<uint64_t> w;
        w.reserve(nb);
        hipLaunchKernelGGL(kSampledWords, dim3(gridFor(nb)), dim3(kTB), 0, st, I.occF.ptr, nb, w.ptr);
        SH_HIP(hipMemcpyAsync(sampledBits, w.ptr, nb * 8, hipMemcpyDeviceToHost, st));
        SH_HIP(hipStreamSynchronize(st));
    }
    if (samples && I.nsamples)
        SH_HIP(hipMemcpyAsync(samples, I.samples.ptr, I.nsamples * 4, hipMemcpyDeviceToHost, st));
    SH_HIP(hipStreamSynchronize(st));
}

}  // namespace sahara
