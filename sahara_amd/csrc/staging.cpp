// staging.cpp — queries and scheme into HBM: the scheme tables of both
// search kernels, the host packers (two bits per symbol with N listed, or
// nibbles; ranks checked), the streamed upload chunk by chunk, and the
// whole-buffer staging of sahara_gpu_stage (search.cpp:111-130, 174-212).
#include <immintrin.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "ctx.h"

namespace sahara {

void packSchemeTable(const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, uint32_t m,
                std::vector<uint32_t>& out, uint32_t& maxErr) {
    if (ns == 0) throw Error("empty search scheme");
    if (m == 0 || m > kMaxPatternLen) throw Error("pattern length out of range");
    out.resize((size_t)ns * m);
    maxErr = 0;
    for (uint32_t s = 0; s < ns; ++s) {
        const uint32_t* P = pi + (size_t)s * m;
        uint32_t lo = P[0], hi = P[0];
        if (P[0] >= m) throw Error("scheme pi out of range");
        for (uint32_t p = 0; p < m; ++p) {
            const uint32_t L = l[(size_t)s * m + p], U = u[(size_t)s * m + p];
            if (L > U || U > kMaxErrors) throw Error("scheme bounds must satisfy l <= u <= 15");
            if (p > 0) {
                if (P[p] == hi + 1) hi = P[p];
                else if (lo > 0 && P[p] == lo - 1) lo = P[p];
                else throw Error("scheme pi is not a connected order (search.cpp:191 expand)");
            }
            maxErr = std::max(maxErr, U);
        }
        for (uint32_t p = 0; p < m; ++p) {
            uint32_t right;
            if (p > 0) right = P[p] > P[p - 1];
            else right = m > 1 ? (P[1] > P[0]) : 1u;
            out[(size_t)s * m + p] = packScheme(P[p], l[(size_t)s * m + p], u[(size_t)s * m + p], right);
        }
    }
}

// Text-phase table, two words per (search, pos):
//   x = packScheme(...) | run << 25 — run = number of consecutive positions
//       from pos (<= 127) on the same side with u == u[pos] and l <= u[pos]:
//       a node at pos with e == u[pos] has no error child anywhere in that
//       run, so the DFS is a forced chain of matches through it;
//   y = a | b << 12 | same << 24 — pattern positions [a, b) covered before
//       step pos; `same` (<= run) positions from pos share pos's l as well,
//       so a chain of matches through them branches the same way at each.
void textTable(const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, uint32_t m,
               const std::vector<uint32_t>& packed, std::vector<uint32_t>& out) {
    out.assign((size_t)ns * m * 2, 0);
    for (uint32_t s = 0; s < ns; ++s) {
        const uint32_t* P = pi + (size_t)s * m;
        const uint32_t* L = l + (size_t)s * m;
        const uint32_t* U = u + (size_t)s * m;
        const uint32_t* Q = packed.data() + (size_t)s * m;
        uint32_t a = P[0], b = P[0];
        for (uint32_t p = 0; p < m; ++p) {
            const uint32_t right = (Q[p] >> 24) & 1u;
            uint32_t run = 1, same = 1;
            while (run < 127 && p + run < m && ((Q[p + run] >> 24) & 1u) == right && U[p + run] == U[p] &&
                   L[p + run] <= U[p])
                ++run;
            while (same < run && L[p + same] == L[p]) ++same;
            out[((size_t)s * m + p) * 2] = Q[p] | (run << 25);
            out[((size_t)s * m + p) * 2 + 1] = a | (b << 12) | (same << 24);
            a = std::min(a, P[p]);
            b = std::max(b, P[p] + 1);
        }
    }
}

// Host pattern bytes -> device, one symbol per byte. Patterns cross PCIe as
// two symbols per byte: host threads each pack a slice, 4 MB at a time, into
// one pinned buffer and queue each piece's DMA as soon as it is packed, and
// kUnpackNibbles expands them on the device. At C3 this halves the 2 GB
// upload, which runs at the link's rate. Returns false when a byte is >= 16
// (no rank of any alphabet; smaller out-of-range ranks are found by the
// device check against this index's sigma).
static bool stageIn(Ctx* c, uint8_t* dst, const uint8_t* src, size_t n) {
    if (const char* e = std::getenv("SAHARA_NIBBLE_UPLOAD")) c->nibbleUpload = std::atoi(e) != 0;
    if (!c->nibbleUpload || n < (64u << 20)) {
        SH_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->st));
        return true;
    }
    const size_t nb = (n + 1) / 2;  // packed bytes
    if (c->nibHostCap < nb) {
        if (c->nibHost) SH_HIP(hipHostFree(c->nibHost));
        c->nibHost = nullptr;
        c->nibHostCap = 0;
        SH_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->nibHost), nb));
        c->nibHostCap = nb;
    }
    c->nibPats.reserve(nb + 8);
    SH_HIP(hipStreamSynchronize(c->st));  // the pinned buffer may still feed the last call's DMA
    uint8_t* out = c->nibHost;
    const unsigned nt = hostThreads(c, 16);
    constexpr size_t kPiece = 4u << 20;
    const size_t pieces = (nb + kPiece - 1) / kPiece;
    std::atomic<uint64_t> orAll{0};
    std::atomic<int> failed{0};
    auto pack = [&](size_t lo, size_t hi) {  // packed bytes [lo, hi)
        uint64_t acc = 0;
        const uint8_t* in = src + 2 * lo;
        const size_t full = std::min(hi, n / 2);  // bytes with both symbols
        size_t i = lo;
        for (; i + 4 <= full; i += 4, in += 8) {  // 8 symbols -> 4 bytes
            uint64_t v;
            std::memcpy(&v, in, 8);
            acc |= v;
            v = (v | (v >> 4)) & 0x00FF00FF00FF00FFull;
            v = (v | (v >> 8)) & 0x0000FFFF0000FFFFull;
            const uint32_t w = (uint32_t)(v | (v >> 16));
            std::memcpy(out + i, &w, 4);
        }
        for (; i < full; ++i, in += 2) {
            out[i] = (uint8_t)(in[0] | (in[1] << 4));
            acc |= (uint64_t)(in[0] | in[1]);
        }
        for (; i < hi; ++i, in += 2) {  // the odd last symbol
            out[i] = in[0];
            acc |= in[0];
        }
        if (acc & 0xF0F0F0F0F0F0F0F0ull) orAll.fetch_or(1, std::memory_order_relaxed);
        if (hipMemcpyAsync(c->nibPats.ptr + lo, out + lo, hi - lo, hipMemcpyHostToDevice, c->st) != hipSuccess)
            failed.store(1);
    };
    auto worker = [&](unsigned t) {  // pieces t, t + nt, ...: the DMA queue fills front to back
        for (size_t k = t; k < pieces; k += nt) pack(k * kPiece, std::min(nb, (k + 1) * kPiece));
    };
    std::vector<std::thread> ts;
    for (unsigned t = 1; t < nt && t < pieces; ++t) ts.emplace_back(worker, t);
    worker(0);
    for (auto& t : ts) t.join();
    if (failed.load()) throw Error("pattern upload failed");
    launchUnpackNibbles(c->nibPats.ptr, dst, n, c->st);
    return orAll.load() == 0;
}

// Any byte of 8 that is no rank of a sigma-letter alphabet (0, or >= sigma;
// ivs::verify_rank, search.cpp:118-120): nonzero high bits. Exact: with every
// byte in [1, 16) the subtraction borrows nowhere and the addition carries
// out of no byte.
static inline uint64_t badRanks8(uint64_t v, uint64_t big) {
    constexpr uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    return (v & 0xF0F0F0F0F0F0F0F0ull) | ((v - ones) & ~v & highs) | ((v + big) & highs);
}

// 2 * count symbols of `in` (one per byte) -> count bytes of `out`, two per
// byte (low nibble first); the bytes from `full` on hold one symbol each (the
// odd last symbol of an upload). Returns nonzero if any symbol is no rank in
// [1, sigma).
static uint64_t packNibblesScalar(const uint8_t* in, uint8_t* out, uint64_t full, uint64_t count, uint32_t sigma) {
    const uint64_t big = (uint64_t)(0x80u - sigma) * 0x0101010101010101ull;
    uint64_t acc = 0, i = 0;
    for (; i + 4 <= full; i += 4, in += 8) {  // 8 symbols -> 4 bytes
        uint64_t v;
        std::memcpy(&v, in, 8);
        acc |= badRanks8(v, big);
        v = (v | (v >> 4)) & 0x00FF00FF00FF00FFull;
        v = (v | (v >> 8)) & 0x0000FFFF0000FFFFull;
        const uint32_t w = (uint32_t)(v | (v >> 16));
        std::memcpy(out + i, &w, 4);
    }
    for (; i < full; ++i, in += 2) {
        out[i] = (uint8_t)(in[0] | (in[1] << 4));
        acc |= (uint64_t)(in[0] == 0 || in[0] >= sigma || in[1] == 0 || in[1] >= sigma);
    }
    for (; i < count; ++i, in += 2) {  // the odd last symbol
        out[i] = in[0];
        acc |= (uint64_t)(in[0] == 0 || in[0] >= sigma);
    }
    return acc;
}

// The same with AVX2, 64 symbols per step: pairs combined by one multiply-add
// (lo * 1 + hi * 16), packed to bytes; ranks checked as max(v - 1, sigma - 2)
// == sigma - 2. About a tenth of the scalar instructions per byte, so that
// 16 host threads pack faster than the GPU searches (the streamed upload).
__attribute__((target("avx2"))) static uint64_t packNibblesAvx2(const uint8_t* in, uint8_t* out, uint64_t full,
                                                                uint64_t count, uint32_t sigma) {
    const __m256i mult = _mm256_set1_epi16(0x1001), one = _mm256_set1_epi8(1);
    const __m256i lim = _mm256_set1_epi8((char)(sigma - 2));
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    for (; i + 32 <= full; i += 32) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + 2 * i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + 2 * i + 32));
        const __m256i ta = _mm256_sub_epi8(a, one), tb = _mm256_sub_epi8(b, one);
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(ta, lim), lim));
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(tb, lim), lim));
        const __m256i pa = _mm256_maddubs_epi16(a, mult), pb = _mm256_maddubs_epi16(b, mult);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i),
                            _mm256_permute4x64_epi64(_mm256_packus_epi16(pa, pb), 0xD8));
    }
    return (uint64_t)!_mm256_testz_si256(bad, bad) |
           packNibblesScalar(in + 2 * i, out + i, full - i, count - i, sigma);
}

// Nonzero if any byte of [p, p + n) is no rank in [1, sigma).
static uint64_t badRanksScalar(const uint8_t* p, uint64_t n, uint32_t sigma) {
    const uint64_t big = (uint64_t)(0x80u - sigma) * 0x0101010101010101ull;
    uint64_t acc = 0, i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v;
        std::memcpy(&v, p + i, 8);
        acc |= badRanks8(v, big);
    }
    for (; i < n; ++i) acc |= (uint64_t)(p[i] == 0 || p[i] >= sigma);
    return acc;
}

__attribute__((target("avx2"))) static uint64_t badRanksAvx2(const uint8_t* p, uint64_t n, uint32_t sigma) {
    const __m256i one = _mm256_set1_epi8(1), lim = _mm256_set1_epi8((char)(sigma - 2));
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i t = _mm256_sub_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i)), one);
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(t, lim), lim));
    }
    return (uint64_t)!_mm256_testz_si256(bad, bad) | badRanksScalar(p + i, n - i, sigma);
}

// Two bits per symbol (SAHARA_UPLOAD_BITS=2, the default for DNA): `count`
// symbols of `in` -> (count + 3) / 4 bytes of `out`, symbol i at bits
// 2 (i % 4) of byte i / 4, coded A C G T = 0 1 2 3. dna5's N (rank 4 of
// sigma 6) is coded 0 and its position (`base` + i) appended to `exc`; the
// device turns the codes straight into both pattern forms and sets the listed
// N positions (kPackFrom2). Returns nonzero if any symbol is no rank in [1, sigma).
uint64_t pack2Scalar(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                            std::vector<uint32_t>& exc) {
    uint64_t bad = 0;
    for (uint64_t i = 0; i < count; i += 4) {
        uint32_t b = 0;
        for (uint32_t q = 0; q < 4 && i + q < count; ++q) {
            const uint32_t r = in[i + q];
            bad |= (uint64_t)(r == 0 || r >= sigma);
            uint32_t code = (r - 1u) & 3u;
            if (sigma == 6 && r >= 4) {
                if (r == 4) exc.push_back((uint32_t)(base + i + q));
                code = r == 5 ? 3u : 0u;
            }
            b |= code << (2 * q);
        }
        out[i / 4] = (uint8_t)b;
    }
    return bad;
}

// The same with AVX2, 128 symbols -> 32 bytes per step: codes t = rank - 1
// (dna5: T 4 -> 3, N 3 -> 0 and listed from a byte mask), pairs combined by
// one multiply-add (t0 + 4 t1), pairs of pairs by another (+ 16), packed to
// bytes and put back in order with one cross-lane permute. The N masks of a
// 16 KB sub-block are kept in a local array and listed after it: a possible
// call (vector growth) inside the vector loop made the compiler spill and
// reload the vector constants and pointers every step (3x slower).
constexpr uint64_t kPackSub = 16384;  // symbols per sub-block

__attribute__((target("avx2"))) uint64_t pack2Avx2(const uint8_t* in, uint8_t* out, uint64_t count,
                                                          uint32_t sigma, uint64_t base, std::vector<uint32_t>& exc) {
    const __m256i one = _mm256_set1_epi8(1), three = _mm256_set1_epi8(3), four = _mm256_set1_epi8(4);
    const __m256i lim = _mm256_set1_epi8((char)(sigma - 2));
    const __m256i m14 = _mm256_set1_epi16(0x0401), m116 = _mm256_set1_epi32(0x00100001);
    const __m256i order = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
    const bool dna5 = sigma == 6;
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    uint32_t nmask[kPackSub / 32], noff[kPackSub / 32];
    while (i + 128 <= count) {
        const uint64_t end = std::min(count & ~uint64_t(127), i + kPackSub);
        uint32_t nn = 0;
        for (; i < end; i += 128) {
            __m256i d[4];
            for (int q = 0; q < 4; ++q) {
                __m256i t = _mm256_sub_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + i + 32 * q)), one);
                bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(t, lim), lim));
                if (dna5) {
                    const __m256i isN = _mm256_cmpeq_epi8(t, three);
                    const uint32_t msk = (uint32_t)_mm256_movemask_epi8(isN);
                    nmask[nn] = msk;
                    noff[nn] = (uint32_t)(i + 32 * q);
                    nn += msk ? 1u : 0u;
                    t = _mm256_andnot_si256(isN, _mm256_add_epi8(t, _mm256_cmpeq_epi8(t, four)));
                }
                t = _mm256_and_si256(t, three);
                d[q] = _mm256_madd_epi16(_mm256_maddubs_epi16(t, m14), m116);
            }
            const __m256i b = _mm256_packus_epi16(_mm256_packus_epi32(d[0], d[1]), _mm256_packus_epi32(d[2], d[3]));
            _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i / 4), _mm256_permutevar8x32_epi32(b, order));
        }
        for (uint32_t k = 0; k < nn; ++k)
            for (uint32_t msk = nmask[k]; msk; msk &= msk - 1u)
                exc.push_back((uint32_t)(base + noff[k] + (uint32_t)__builtin_ctz(msk)));
    }
    return (uint64_t)!_mm256_testz_si256(bad, bad) | pack2Scalar(in + i, out + i / 4, count - i, sigma, base + i, exc);
}

// The same with AVX-512 (BW), 64 symbols -> 16 bytes per step: rank checks
// and the N / T recoding in mask registers, the four codes of a byte combined
// by the same two multiply-adds, and the dwords narrowed to bytes in order
// (vpmovdb). N masks listed per sub-block as above.
__attribute__((target("avx512f,avx512bw"))) uint64_t pack2Avx512(const uint8_t* in, uint8_t* out, uint64_t count,
                                                                 uint32_t sigma, uint64_t base,
                                                                 std::vector<uint32_t>& exc) {
    const __m512i one = _mm512_set1_epi8(1), three = _mm512_set1_epi8(3), four = _mm512_set1_epi8(4);
    const __m512i lim = _mm512_set1_epi8((char)(sigma - 2));
    const __m512i m14 = _mm512_set1_epi16(0x0401), m116 = _mm512_set1_epi32(0x00100001);
    const bool dna5 = sigma == 6;
    __mmask64 bad = 0;
    uint64_t i = 0;
    uint64_t nmask[kPackSub / 64];
    uint32_t noff[kPackSub / 64];
    while (i + 64 <= count) {
        const uint64_t end = std::min(count & ~uint64_t(63), i + kPackSub);
        uint32_t nn = 0;
        for (; i < end; i += 64) {
            __m512i t = _mm512_sub_epi8(_mm512_loadu_si512(reinterpret_cast<const void*>(in + i)), one);
            bad |= _mm512_cmpgt_epu8_mask(t, lim);
            if (dna5) {
                const __mmask64 isN = _mm512_cmpeq_epi8_mask(t, three);
                nmask[nn] = (uint64_t)isN;
                noff[nn] = (uint32_t)i;
                nn += isN ? 1u : 0u;
                t = _mm512_mask_sub_epi8(t, _mm512_cmpeq_epi8_mask(t, four), t, one);  // T 4 -> 3
                t = _mm512_maskz_mov_epi8(~isN, t);                                   // N 3 -> 0
            }
            t = _mm512_and_si512(t, three);
            const __m512i d = _mm512_madd_epi16(_mm512_maddubs_epi16(t, m14), m116);
            _mm_storeu_si128(reinterpret_cast<__m128i*>(out + i / 4), _mm512_cvtepi32_epi8(d));
        }
        for (uint32_t k = 0; k < nn; ++k)
            for (uint64_t msk = nmask[k]; msk; msk &= msk - 1u)
                exc.push_back((uint32_t)(base + noff[k] + (uint32_t)__builtin_ctzll(msk)));
    }
    return (uint64_t)(bad != 0) | pack2Avx2(in + i, out + i / 4, count - i, sigma, base + i, exc);
}

bool hostHasAvx2() {
    static const bool has = __builtin_cpu_supports("avx2");
    return has;
}

bool hostHasAvx512() {
    static const bool has = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512f");
    return has;
}

uint64_t pack2Best(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                   std::vector<uint32_t>& exc) {
    if (hostHasAvx512()) return pack2Avx512(in, out, count, sigma, base, exc);
    if (hostHasAvx2()) return pack2Avx2(in, out, count, sigma, base, exc);
    return pack2Scalar(in, out, count, sigma, base, exc);
}

TaskPool& hostPool(Ctx* c) {
    // The packing threads read the caller's reads wherever their pages are,
    // so they stay unbound (SAHARA_PACK_BIND=1: on the GPU's node like the
    // context's other threads). Measured on the GPU box (2 NUMA nodes, 16 CPUs
    // of quota; tools/probe/pack_bench numa): 16 threads bound to the GPU's
    // node pack 250 GB/s of input on that node but 65 GB/s of input on the
    // other; unbound they pack 194-210 GB/s either way.
    // (SAHARA_PACK_THREADS: packing threads, default 16; read per call, the
    // pool is rebuilt when it changes)
    unsigned cap = 16;
    if (const char* t = std::getenv("SAHARA_PACK_THREADS")) cap = (unsigned)std::max(1, std::min(64, std::atoi(t)));
    // SAHARA_PACK_BIND=1: the GPU's node, else unbound (binding to the node
    // that holds the call's reads measured slower inside the call: 539M
    // against 592M reads/s, profiles/r03_pcie_compact_dma.txt)
    const char* e = std::getenv("SAHARA_PACK_BIND");
    const int node = e && std::atoi(e) == 1 ? c->place.node : -1;
    if (!c->pool || c->poolCap != cap || c->poolNode != node) {
        drainPacking(c);
        c->pool.reset();
        c->packPlace = placementOfNode(node);
        c->pool = std::make_unique<TaskPool>(std::min(cap, c->packPlace.ncpus > 0 ? (unsigned)c->packPlace.ncpus : cap),
                                             node >= 0 ? &c->packPlace : nullptr);
        c->poolCap = cap;
        c->poolNode = node;
    }
    return *c->pool;
}

// f(k) for k in [0, n) on the pool's threads; returns when all are done
static void runPieces(TaskPool& P, uint64_t n, const std::function<void(uint64_t)>& f) {
    TaskGroup g;
    g.begin(n);
    std::vector<std::function<void()>> fs;
    fs.reserve(n);
    for (uint64_t k = 0; k < n; ++k)
        fs.emplace_back([&f, &g, k] {
            f(k);
            g.oneDone();
        });
    P.postMany(fs);
    g.wait();
}

// An index image's arrays go up through the pinned ring: the pool's threads
// copy one slot's worth of the source at a time (a mapped .idx faults its
// pages in on all of them), and the copy engine moves each slot while the next
// one fills. A pageable hipMemcpyAsync is staged by the runtime on the calling
// thread alone.
void uploadViaRing(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (c->ringInit.joinable()) c->ringInit.join();
    if (!c->ring || bytes < Ctx::kRingSlot) {
        SH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
        return;
    }
    TaskPool& P = hostPool(c);
    constexpr size_t kPiece = 1u << 20;  // bytes per pool task
    const uint8_t* s = static_cast<const uint8_t*>(src);
    for (size_t off = 0; off < bytes; off += Ctx::kRingSlot) {
        const size_t slot = (size_t)(c->ringLoadNext++ % Ctx::kRingSlots);
        const size_t len = std::min(Ctx::kRingSlot, bytes - off);
        SH_HIP(hipEventSynchronize(c->ringEv[slot]));  // the slot's previous copy is done
        uint8_t* stage = c->ring + slot * Ctx::kRingSlot;
        runPieces(P, (len + kPiece - 1) / kPiece, [&](uint64_t i) {
            std::memcpy(stage + i * kPiece, s + off + i * kPiece, std::min(kPiece, len - i * kPiece));
        });
        SH_HIP(hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, stage, len, hipMemcpyHostToDevice, st));
        SH_HIP(hipEventRecord(c->ringEv[slot], st));
    }
}

static uint64_t chunkCount(const Ctx::Upload& U) { return U.chunk ? (U.rows + U.chunk - 1) / U.chunk : 0; }

// Posts the 2-bit packing of chunk j (the next one not yet posted) to the
// pool: its pieces pack into ring slot j % kRingSlots, each piece listing its
// N positions. The slot's previous DMA (chunk j - kRingSlots) must be done.
static void submitPack(Ctx* c, uint64_t j) {
    Ctx::Upload& U = c->up;
    const size_t slot = (size_t)(j % Ctx::kRingSlots);
    Ctx::PackJob& J = c->packJobs[slot];
    J.group.wait();  // (finished by its uploadChunk already; never blocks)
    if (!(U.prepacked && U.srcPinned)) SH_HIP(hipEventSynchronize(c->ringEv[slot]));  // (pinned codes: no ring)
    const uint32_t m = c->m, sigma = c->I.sigma;
    const uint64_t r0 = j * U.chunk, r1 = std::min(U.rows, r0 + U.chunk);
    const uint64_t s0 = r0 * m, n = (r1 - r0) * m;
    // symbols per piece (SAHARA_PACK_PIECE, a multiple of 4; 4M: 1 MB packed)
    uint64_t pieceSyms = 4u << 20;
    if (const char* e = std::getenv("SAHARA_PACK_PIECE")) pieceSyms = std::max<uint64_t>(4096, std::atoll(e)) & ~uint64_t(3);
    J.chunk = j;
    J.pieceSyms = pieceSyms;
    J.bad.store(0, std::memory_order_relaxed);
    uint8_t* out = c->ring + slot * Ctx::kRingSlot;
    std::vector<std::function<void()>> fs;
    if (U.prepacked) {  // codes as given: the chunk's bytes of the caller's buffer, copied in pieces
        const uint64_t B0 = (U.sym0 + s0) / 4, nb = (U.sym0 + s0 + n + 3) / 4 - B0, pb = pieceSyms / 4;
        J.pieces = U.srcPinned ? 0 : (nb + pb - 1) / pb;  // pinned: the DMA reads the caller's buffer
        J.group.begin(J.pieces);
        const uint8_t* src = U.src + B0;
        fs.reserve(J.pieces);
        for (uint64_t k = 0; k < J.pieces; ++k)
            fs.emplace_back([&J, out, src, nb, pb, k] {
                const uint64_t lo = k * pb, hi = std::min(nb, lo + pb);
                std::memcpy(out + lo, src + lo, hi - lo);
                J.group.oneDone();
            });
    } else {
        J.pieces = (n + pieceSyms - 1) / pieceSyms;
        if (J.exc.size() < J.pieces) J.exc.resize(J.pieces);
        for (auto& v : J.exc) v.clear();
        J.group.begin(J.pieces);
        const uint8_t* src = U.src + s0;
        fs.reserve(J.pieces);
        for (uint64_t k = 0; k < J.pieces; ++k)
            fs.emplace_back([&J, out, src, n, sigma, k] {
                const uint64_t lo = k * J.pieceSyms, hi = std::min(n, lo + J.pieceSyms);
                if (pack2Best(src + lo, out + lo / 4, hi - lo, sigma, lo, J.exc[k])) J.bad.store(1, std::memory_order_relaxed);
                J.group.oneDone();
            });
    }
    hostPool(c).postMany(fs);
    U.submitted = j + 1;
    c->mark("pack posted", j);
}

// Keeps the next U.ahead chunks after the last enqueued one posted to the
// pool (2-bit upload), within the ring's slots.
static void packAhead(Ctx* c) {
    Ctx::Upload& U = c->up;
    if (!c->streaming || U.bits != 2 || U.bad) return;
    const uint64_t doneChunks = U.done / U.chunk + (U.done % U.chunk ? 1 : 0);
    const uint64_t want = std::min({chunkCount(U), doneChunks + U.ahead, doneChunks + Ctx::kRingSlots - 1});
    while (U.submitted < want) submitPack(c, U.submitted);
}

void drainPacking(Ctx* c) {
    for (auto& J : c->packJobs) J.group.wait();
}

// H2D copy of one chunk's staged bytes on stE (SAHARA_TIMING=2: timed with
// events; splitting a chunk over 2-4 streams measured no faster,
// profiles/r03_pcie_upload_streams.txt)
static void uploadCopy(Ctx* c, void* dst, const void* src, uint64_t bytes) {
    if (c->traceOn) {  // the DMA's own duration (printed with the marks)
        if (c->dmaUsed == c->dmaEv.size()) {
            hipEvent_t a, b;
            SH_HIP(hipEventCreate(&a));
            SH_HIP(hipEventCreate(&b));
            c->dmaEv.push_back({0, {a, b}});
        }
        auto& d = c->dmaEv[c->dmaUsed++];
        d.first = bytes;
        SH_HIP(hipEventRecord(d.second.first, c->stE));
        SH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stE));
        SH_HIP(hipEventRecord(d.second.second, c->stE));
        return;
    }
    SH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stE));
}

// Enqueues the next chunk of the streamed upload (Ctx::Upload): packed on the
// host into its ring slot (2 bits: posted ahead by packAhead, waited for
// here), its DMA on stE (nothing else: the DMAs run back to back at the link's
// rate) and, on stream `kst` after the DMA's event, the unpack (and
// reverse-complement interleave) kernel and both pattern packings. A chunk
// with a byte that is no rank sets up.bad and enqueues nothing.
void uploadChunk(Ctx* c, hipStream_t kst) {
    Ctx::Upload& U = c->up;
    const auto t0 = std::chrono::steady_clock::now();
    c->mark("pack", U.done / std::max<uint64_t>(U.chunk, 1));
    const uint64_t r0 = U.done, r1 = std::min(U.rows, r0 + U.chunk);
    const uint32_t m = c->m, sigma = c->I.sigma;
    const uint64_t s0 = r0 * m, s1 = r1 * m, nsym = U.rows * m;  // symbols
    uint8_t* raw = U.rc ? c->readRaw.ptr : c->rawPats.ptr;
    TaskPool& P = hostPool(c);
    std::atomic<int> bad{0};
    constexpr uint64_t kPiece = 1u << 20;
    const bool avx2 = hostHasAvx2();
    const uint64_t j = r0 / U.chunk;
    const size_t slot = (size_t)(j % Ctx::kRingSlots);
    // a chunk owns bytes [s0 / 2, (s1 + 1) / 2) of the ring slot and of the
    // device staging buffer at any encoding (s0 is even)
    const uint64_t b0 = s0 / 2, b1 = (s1 + 1) / 2;
    uint32_t bits = U.bits;
    uint64_t nExc = 0, excOff = 0;  // 2 bits: the N list, at byte excOff of the chunk's region
    const uint32_t* excDev = nullptr;  // ... on the device
    uint32_t so = 0;                   // read r0's first symbol in the chunk's first byte (prepacked)
    uint8_t* out = c->ring + slot * Ctx::kRingSlot;
    if (bits == 2 && U.prepacked) {
        if (U.submitted <= j) submitPack(c, j);
        c->packJobs[slot].group.wait();
        c->mark("slot free", j);
        const uint64_t S0 = U.sym0 + s0, S1 = U.sym0 + s1;
        so = (uint32_t)(S0 & 3u);
        nExc = U.nFirst[j + 1] - U.nFirst[j];
        excDev = c->nList.ptr + U.nFirst[j];
        uploadCopy(c, c->nibPats.ptr + b0, U.srcPinned ? U.src + S0 / 4 : out, (S1 + 3) / 4 - S0 / 4);
        c->mark("dma enqueued", j);
    } else if (bits == 2) {
        if (U.submitted <= j) submitPack(c, j);  // (U.submitted == j: chunks post in order)
        Ctx::PackJob& J = c->packJobs[slot];
        J.group.wait();
        c->mark("slot free", j);
        if (J.bad.load(std::memory_order_relaxed)) bad.store(1);
        const uint64_t n = s1 - s0;
        for (uint64_t k = 0; k < J.pieces; ++k) nExc += J.exc[k].size();
        c->mark("pack cpu done", j);
        excOff = ((b0 + (n + 3) / 4 + 3) & ~uint64_t(3)) - b0;  // 4-aligned on the device
        if (excOff + 4 * nExc > b1 - b0) {
            bits = 4;  // N-rich chunk: the list would not fit, go as nibbles
        } else if (!bad.load()) {
            // the pieces' lists, concatenated in piece order, are sorted
            uint8_t* e = out + excOff;
            for (uint64_t k = 0; k < J.pieces; ++k) {
                const auto& v = J.exc[k];
                if (!v.empty()) std::memcpy(e, v.data(), v.size() * 4);
                e += v.size() * 4;
            }
            uploadCopy(c, c->nibPats.ptr + b0, out, excOff + 4 * nExc);
            excDev = reinterpret_cast<const uint32_t*>(c->nibPats.ptr + b0 + excOff);
            c->mark("dma enqueued", j);
        }
    } else {
        SH_HIP(hipEventSynchronize(c->ringEv[slot]));  // the slot's previous DMA is done
        c->mark("slot free", j);
    }
    if (bits == 4 && !bad.load()) {
        const uint64_t pieces = (b1 - b0 + kPiece - 1) / kPiece;
        runPieces(P, pieces, [&](uint64_t k) {
            const uint64_t lo = b0 + k * kPiece, hi = std::min(b1, lo + kPiece);
            const uint64_t full = std::min(hi, std::max(lo, nsym / 2)) - lo;  // bytes with two symbols
            const uint8_t* in = U.src + 2 * lo;
            const uint64_t acc = avx2 ? packNibblesAvx2(in, out + (lo - b0), full, hi - lo, sigma)
                                      : packNibblesScalar(in, out + (lo - b0), full, hi - lo, sigma);
            if (acc) bad.store(1, std::memory_order_relaxed);
        });
        if (!bad.load()) uploadCopy(c, c->nibPats.ptr + b0, out, b1 - b0);
    } else if (bits == 8) {  // one byte per symbol (SAHARA_UPLOAD_BITS=8): check, then copy as given
        const uint64_t pieces = (s1 - s0 + kPiece - 1) / kPiece;
        runPieces(P, pieces, [&](uint64_t k) {
            const uint64_t lo = s0 + k * kPiece, hi = std::min(s1, lo + kPiece);
            const uint64_t acc = avx2 ? badRanksAvx2(U.src + lo, hi - lo, sigma) : badRanksScalar(U.src + lo, hi - lo, sigma);
            if (acc) bad.store(1, std::memory_order_relaxed);
        });
        if (!bad.load()) SH_HIP(hipMemcpyAsync(raw + s0, U.src + s0, s1 - s0, hipMemcpyHostToDevice, c->stE));
    }
    U.hostMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (bad.load()) {
        U.bad = true;
        return;
    }
    SH_HIP(hipEventRecord(c->ringEv[slot], c->stE));  // the chunk's DMA
    SH_HIP(hipStreamWaitEvent(kst, c->ringEv[slot], 0));
    if (bits == 4) launchUnpackNibbles(c->nibPats.ptr + b0, raw + s0, s1 - s0, kst);
    U.chunks[bits == 2 ? 0 : bits == 4 ? 1 : 2]++;
    const uint64_t p0 = U.rc ? 2 * r0 : r0, p1 = U.rc ? std::min(2 * r1, c->npat) : r1;
    if (bits == 2) {  // straight into both pattern forms (no byte pass)
        launchPackFrom2(c->nibPats.ptr + b0, so, excDev, (uint32_t)nExc, r0, p0, p1, m, U.rc, sigma, c->patWords,
                        c->patBlocks, c->pats.ptr + 0, c->pats3.ptr + 0, kst);
        U.done = r1;
        c->mark("packed", r0 / U.chunk);
        return;
    }
    if (U.rc) launchInterleaveRC(c->readRaw.ptr, r0, r1, m, sigma, c->npat, c->rawPats.ptr, kst);
    if (p1 > p0) {
        launchPackPatterns(c->rawPats.ptr + p0 * m, p1 - p0, m, c->patWords, sigma, c->pats.ptr + p0 * c->patWords,
                           c->badFlag.ptr, kst);
        launchPackPatterns3(c->rawPats.ptr + p0 * m, p1 - p0, m, c->patBlocks, c->pats3.ptr + p0 * c->patBlocks, kst);
    }
    U.done = r1;
    c->mark("packed", r0 / U.chunk);
}

// Streamed upload: makes sure the patterns [0, patEnd) are enqueued, their
// device-side packing on stream kst (a no-op when the patterns were staged
// whole).
void ensureUploaded(Ctx* c, uint64_t patEnd, hipStream_t kst) {
    if (!c->streaming) return;
    Ctx::Upload& U = c->up;
    auto covered = [&] { return U.rc ? std::min(2 * U.done, c->npat) : U.done; };
    while (covered() < patEnd) {
        uploadChunk(c, kst);
        if (U.bad) {
            drainPacking(c);  // chunks posted ahead still read the caller's buffer
            throw Error("pattern rank out of range for this index");
        }
    }
    packAhead(c);  // the pool packs the next chunks while this batch searches
}

// The scheme half of staging: host tables, their upload, the k-mer starts.
void stageScheme(Ctx* c, uint64_t npat, uint32_t m, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                 uint32_t ns, int edit) {
    if (npat == 0) throw Error("no patterns");
    std::vector<uint32_t> packed, cover;
    packSchemeTable(pi, l, u, ns, m, packed, c->maxErr);
    if ((size_t)ns * m * 4 > 60 * 1024) throw Error("scheme too large for LDS (searches * len > 15360)");
    if (ns > 255) throw Error("at most 255 searches per scheme");
    textTable(pi, l, u, ns, m, packed, cover);
    c->scheme.reserve(packed.size());
    SH_HIP(hipMemcpyAsync(c->scheme.ptr, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, c->st));
    c->cover.reserve(cover.size());
    SH_HIP(hipMemcpyAsync(c->cover.ptr, cover.data(), cover.size() * 4, hipMemcpyHostToDevice, c->st));
    // searches whose first kmerK steps admit no error start from the k-mer table
    std::vector<uint32_t> kst(ns, 0xFFFFFFFFu);
    const uint32_t K = c->I.kmerK;
    for (uint32_t s = 0; K && K <= m && s < ns; ++s) {
        bool exact = true;
        uint32_t lo = pi[(size_t)s * m];
        for (uint32_t p = 0; p < K; ++p) {
            exact = exact && u[(size_t)s * m + p] == 0;
            lo = std::min(lo, pi[(size_t)s * m + p]);
        }
        if (exact) kst[s] = lo;
    }
    c->kmerStart.reserve(ns);
    SH_HIP(hipMemcpyAsync(c->kmerStart.ptr, kst.data(), ns * 4, hipMemcpyHostToDevice, c->st));
    SH_HIP(hipStreamSynchronize(c->st));
    c->nsearch = ns;
    c->edit = edit != 0;
}

// Staging for a streamed search: the scheme now, the patterns chunk by chunk
// during the pass (uploadChunk). src holds `rows` rows of m symbols: the
// patterns, or (rc) the reads whose interleave with their reverse
// complements, cut to npat, is the query list.
// Reads given two bits per symbol: their N positions (stream positions,
// ascending) checked and uploaded once per call, each relative to the first
// whole byte of its chunk, chunk j's from entry U.nFirst[j] (kPackFrom2 sets
// them). Every 2-bit code is an A, C, G or T: nothing else to check.
static void stagePackedN(Ctx* c, const PackedReads& P, uint64_t rows, uint32_t m) {
    Ctx::Upload& U = c->up;
    U.prepacked = true;
    U.sym0 = P.sym0;
    // codes in page-locked memory (sahara_host_alloc, sahara_read_fasta's
    // form 2, or the caller's own) go up by DMA straight from there
    auto pinned = [](const void* p) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, p) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return at.type == hipMemoryTypeHost && at.hostPointer != nullptr;
    };
    const uint64_t b0 = P.sym0 / 4, b1 = (P.sym0 + rows * m + 3) / 4;
    U.srcPinned = pinned(U.src + b0) && pinned(U.src + b1 - 1);
    const uint64_t lo = P.sym0, hi = P.sym0 + rows * m;
    const uint64_t* all = P.nCount ? P.nPos : nullptr;
    // the whole list, not only this call's range: the binary searches below
    // place the range correctly only in an ascending list (a shard of a larger
    // stream sees every entry). Checked once per list (a stream's shards share
    // it); the range found is checked on every call.
    const char* kUnordered = "N positions of packed reads must be strictly ascending";
    if (all && (c->nPosChecked != all || c->nCountChecked != P.nCount)) {
        for (uint64_t i = 1; i < P.nCount; ++i)
            if (all[i] <= all[i - 1]) throw Error(kUnordered);
        c->nPosChecked = all;
        c->nCountChecked = P.nCount;
    }
    const uint64_t* b = all ? std::lower_bound(all, all + P.nCount, lo) : nullptr;
    const uint64_t* e = all ? std::lower_bound(b, all + P.nCount, hi) : nullptr;
    if (all) {  // [b, e) ascending inside [lo, hi), its neighbours outside
        const uint64_t* end = all + P.nCount;
        if ((b > all && b[-1] >= lo) || (e < end && *e < hi)) throw Error(kUnordered);
        for (const uint64_t* q = b; q < e; ++q)
            if (*q < lo || *q >= hi || (q > b && *q <= q[-1])) throw Error(kUnordered);
    }
    const uint64_t nN = all ? (uint64_t)(e - b) : 0;
    if (nN && c->I.sigma == 5) throw Error("pattern rank out of range for this index");  // N is no dna4 rank
    const uint64_t nch = chunkCount(U);
    U.nFirst.assign(nch + 1, nN);
    std::vector<uint32_t> rel(nN);
    uint64_t i = 0;
    for (uint64_t j = 0; j < nch; ++j) {
        const uint64_t S0 = lo + j * U.chunk * m, S1 = lo + std::min(rows, (j + 1) * U.chunk) * m;
        U.nFirst[j] = i;
        for (; i < nN && b[i] < S1; ++i) rel[i] = (uint32_t)(b[i] - (S0 & ~uint64_t(3)));
    }
    c->nList.reserve(std::max<uint64_t>(nN, 1));
    if (nN) SH_HIP(hipMemcpy(c->nList.ptr, rel.data(), nN * 4, hipMemcpyHostToDevice));
}

// src holds `rows` rows of m symbols: the patterns, or (rc) the reads whose
// interleave with their reverse complements, cut to npat, is the query list;
// one rank per byte, or (packed) two bits per symbol with the N positions
// listed (the reads of sahara_gpu_search_packed[_compact]).
void stageStreamed(Ctx* c, const uint8_t* src, uint64_t rows, bool rc, uint64_t npat, uint32_t m,
                   const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, int edit,
                   const PackedReads* packed) {
    c->staged = c->streaming = false;
    if (m == 0 || m > kMaxPatternLen) throw Error("pattern length out of range");
    if (packed && c->I.sigma != 5 && c->I.sigma != 6) throw Error("reads two bits per symbol need a dna4 or dna5 index");
    stageScheme(c, npat, m, pi, l, u, ns, edit);
    c->m = m;
    c->npat = npat;
    c->patWords = (m + 7) / 8;
    c->patBlocks = (m + 31) / 32;
    c->rawPats.reserve(npat * m);
    c->pats.reserve(npat * c->patWords + 4);  // + tail words read by paired loads
    c->pats3.reserve(npat * c->patBlocks);
    if (rc) c->readRaw.reserve(rows * m);
    c->badFlag.reserve(1);
    drainPacking(c);  // (a failed call drained already)
    Ctx::Upload& U = c->up;
    U = Ctx::Upload{};
    if (const char* e = std::getenv("SAHARA_PACK_AHEAD")) U.ahead = (uint32_t)std::max(0, std::atoi(e));
    c->dmaUsed = 0;
    U.src = src;
    U.rc = rc;
    U.rows = rows;
    // symbols cross PCIe at 2 bits (DNA: A C G T codes, N positions listed),
    // 4 bits (any alphabet) or 8 (as given): SAHARA_UPLOAD_BITS, or
    // SAHARA_NIBBLE_UPLOAD=0 for 8
    if (const char* e = std::getenv("SAHARA_NIBBLE_UPLOAD")) c->nibbleUpload = std::atoi(e) != 0;
    U.bits = !c->nibbleUpload ? 8u : (c->I.sigma == 5 || c->I.sigma == 6) ? 2u : 4u;
    if (const char* e = std::getenv("SAHARA_UPLOAD_BITS")) {
        const int b = std::atoi(e);
        if (b == 2 || b == 4 || b == 8) U.bits = (uint32_t)b;
    }
    if (U.bits == 2 && c->I.sigma != 5 && c->I.sigma != 6) U.bits = 4;
    if (packed) U.bits = 2;
    // 1M patterns per chunk (SAHARA_UPLOAD_CHUNK), at most one ring slot of nibbles
    uint64_t chunkPats = 1u << 20;
    if (const char* e = std::getenv("SAHARA_UPLOAD_CHUNK")) chunkPats = std::max<uint64_t>(2, std::atoll(e));
    uint64_t chunk = rc ? chunkPats / 2 : chunkPats;
    if (U.bits != 8) chunk = std::min<uint64_t>(chunk, Ctx::kRingSlot * 2 / m);
    // a call of fewer than four chunks is cut in four, so that its first
    // batch's seeds and text phase start on a quarter of the upload (C2: 1M
    // reads, one batch; pass.cpp seeds the first batch chunk by chunk)
    chunk = std::min<uint64_t>(chunk, std::max<uint64_t>(1, (rows + 3) / 4));
    // chunk * m a multiple of 32 symbols: every chunk's region of the staging
    // buffers (s0 / 2 bytes at 2 or 4 bits, s0 at 8) then starts 16-B aligned
    // for kPackFrom2's word loads (C5: m = 250)
    uint64_t g = 32;
    while (m % g) g /= 2;
    const uint64_t step = std::max<uint64_t>(2, 32 / g);
    U.chunk = std::max<uint64_t>(step, chunk - chunk % step);
    if (packed) stagePackedN(c, *packed, rows, m);
    if (c->ringInit.joinable()) c->ringInit.join();
    if (U.bits != 8 && !c->ring) throw Error("could not pin the upload ring buffer");
    for (hipEvent_t e : c->ringEv) SH_HIP(hipEventSynchronize(e));  // the last call's DMAs
    if (U.bits != 8) c->nibPats.reserve((rows * m + 1) / 2 + 16);  // + the 12 B the 2-bit packer's last loads may touch
    SH_HIP(hipMemsetAsync(c->badFlag.ptr, 0, sizeof(uint32_t), c->stE));
    c->stageMs = 0;
    c->staged = c->streaming = true;
}

void stage(Ctx* c, const uint8_t* ranks, uint64_t npat, uint32_t m, const uint32_t* pi, const uint32_t* l,
           const uint32_t* u, uint32_t ns, int edit) {
    if (npat == 0) throw Error("no patterns");
    c->staged = c->streaming = false;
    std::vector<uint32_t> packed;
    packSchemeTable(pi, l, u, ns, m, packed, c->maxErr);  // a bad scheme fails before the upload
    if ((size_t)ns * m * 4 > 60 * 1024) throw Error("scheme too large for LDS (searches * len > 15360)");
    if (ns > 255) throw Error("at most 255 searches per scheme");
    const auto t0 = std::chrono::steady_clock::now();
    c->patWords = (m + 7) / 8;
    {
        DevBuf<uint8_t>& raw = c->rawPats;  // kept: no 2 GB allocate / free per call at C3
        raw.reserve(npat * m);
        if (!stageIn(c, raw.ptr, ranks, npat * m)) {
            c->staged = false;
            throw Error("pattern rank out of range for this index");
        }
        c->pats.reserve(npat * c->patWords + 4);  // + tail words read by paired loads
        SH_HIP(hipMemsetAsync(c->small.ptr, 0, sizeof(uint32_t), c->st));
        launchPackPatterns(raw.ptr, npat, m, c->patWords, c->I.sigma, c->pats.ptr, c->small.ptr, c->st);
        c->patBlocks = (m + 31) / 32;
        c->pats3.reserve(npat * c->patBlocks);
        launchPackPatterns3(raw.ptr, npat, m, c->patBlocks, c->pats3.ptr, c->st);
        uint32_t bad = 0;
        SH_HIP(hipMemcpyAsync(&bad, c->small.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost, c->st));
        SH_HIP(hipStreamSynchronize(c->st));
        if (bad) {
            c->staged = false;
            throw Error("pattern rank out of range for this index");
        }
    }
    stageScheme(c, npat, m, pi, l, u, ns, edit);
    c->npat = npat;
    c->m = m;
    c->staged = true;
    c->stageMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace sahara
