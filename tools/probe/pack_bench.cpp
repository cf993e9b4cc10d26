// Host packing throughput probe for the streamed upload (staging.cpp
// pack2Avx2 / pack2Avx512): 1 GB of dna5 ranks packed to 2 bits per symbol
// by T threads, with and without software prefetch, AVX2 and AVX-512.
// Build: hipcc -O3 -std=c++17 -pthread tools/probe/pack_bench.cpp -o tools/probe/pack_bench
// (`pack_bench <MB> numa [pinned]`: NUMA cases; pinned = the output in
// hipHostMalloc memory like the library's upload ring)
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

template <bool PF>
__attribute__((target("avx2"))) uint64_t pack2(const uint8_t* in, uint8_t* out, uint64_t count) {
    const __m256i one = _mm256_set1_epi8(1), three = _mm256_set1_epi8(3), four = _mm256_set1_epi8(4);
    const __m256i lim = _mm256_set1_epi8(4);
    const __m256i m14 = _mm256_set1_epi16(0x0401), m116 = _mm256_set1_epi32(0x00100001);
    const __m256i order = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
    __m256i bad = _mm256_setzero_si256();
    uint64_t nN = 0;
    for (uint64_t i = 0; i + 128 <= count; i += 128) {
        if (PF) _mm_prefetch(reinterpret_cast<const char*>(in + i + 2048), _MM_HINT_T0),
                _mm_prefetch(reinterpret_cast<const char*>(in + i + 2048 + 64), _MM_HINT_T0);
        __m256i d[4];
        for (int q = 0; q < 4; ++q) {
            __m256i t = _mm256_sub_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + i + 32 * q)), one);
            bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(t, lim), lim));
            const __m256i isN = _mm256_cmpeq_epi8(t, three);
            nN += (uint64_t)__builtin_popcount((uint32_t)_mm256_movemask_epi8(isN));
            t = _mm256_andnot_si256(isN, _mm256_add_epi8(t, _mm256_cmpeq_epi8(t, four)));
            t = _mm256_and_si256(t, three);
            d[q] = _mm256_madd_epi16(_mm256_maddubs_epi16(t, m14), m116);
        }
        const __m256i b = _mm256_packus_epi16(_mm256_packus_epi32(d[0], d[1]), _mm256_packus_epi32(d[2], d[3]));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i / 4), _mm256_permutevar8x32_epi32(b, order));
    }
    return nN + (uint64_t)!_mm256_testz_si256(bad, bad);
}

template <bool PF>
__attribute__((target("avx512f,avx512bw"))) uint64_t pack512(const uint8_t* in, uint8_t* out, uint64_t count) {
    const __m512i one = _mm512_set1_epi8(1), three = _mm512_set1_epi8(3), four = _mm512_set1_epi8(4);
    const __m512i lim = _mm512_set1_epi8(4);
    const __m512i m14 = _mm512_set1_epi16(0x0401), m116 = _mm512_set1_epi32(0x00100001);
    __mmask64 bad = 0;
    uint64_t nN = 0;
    for (uint64_t i = 0; i + 64 <= count; i += 64) {
        if (PF) _mm_prefetch(reinterpret_cast<const char*>(in + i + 2048), _MM_HINT_T0);
        __m512i t = _mm512_sub_epi8(_mm512_loadu_si512(reinterpret_cast<const void*>(in + i)), one);
        bad |= _mm512_cmpgt_epu8_mask(t, lim);
        const __mmask64 isN = _mm512_cmpeq_epi8_mask(t, three);
        nN += (uint64_t)__builtin_popcountll((uint64_t)isN);
        t = _mm512_mask_sub_epi8(t, _mm512_cmpeq_epi8_mask(t, four), t, one);
        t = _mm512_maskz_mov_epi8(~isN, t);
        t = _mm512_and_si512(t, three);
        const __m512i d = _mm512_madd_epi16(_mm512_maddubs_epi16(t, m14), m116);
        _mm_storeu_si128(reinterpret_cast<__m128i*>(out + i / 4), _mm512_cvtepi32_epi8(d));
    }
    return nN + (bad != 0);
}

static void bindTo(int node) {  // GPU box: node 0 = CPUs 0-63, node 1 = 64-127 (+ SMT siblings 128-255)
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c = 0; c < 64; ++c) {
        CPU_SET(node * 64 + c, &set);
        CPU_SET(128 + node * 64 + c, &set);
    }
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

// The library's pattern: T threads bound to `packNode` take 4 MB pieces round
// robin, input first touched by a thread on `dataNode`.
static bool g_pinned = false;
static void numaCase(uint64_t n, int dataNode, int packNode, unsigned T) {
    uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    std::thread([&] {
        bindTo(dataNode);
        in = static_cast<uint8_t*>(std::malloc(n));
        if (g_pinned) {
            void* p = nullptr;
            if (hipHostMalloc(&p, n / 4 + 64, hipHostMallocPortable) != hipSuccess) std::abort();
            out = static_cast<uint8_t*>(p);
        } else {
            out = static_cast<uint8_t*>(std::malloc(n / 4 + 64));
        }
        std::mt19937_64 g(1);
        const uint8_t code[4] = {1, 2, 3, 5};
        for (uint64_t i = 0; i < n; i += 32) {
            uint64_t x = g();
            for (int j = 0; j < 32 && i + j < n; ++j) in[i + j] = code[(x >> (2 * j)) & 3];
        }
        std::memset(out, 0, n / 4 + 64);
    }).join();
    const uint64_t piece = 4u << 20, np = (n + piece - 1) / piece;
    double best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
        std::vector<std::thread> th;
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                if (packNode >= 0) bindTo(packNode);
                for (uint64_t k = t; k < np; k += T) {
                    const uint64_t b = k * piece, e = std::min(n, b + piece);
                    volatile uint64_t r = pack512<false>(in + b, out + b / 4, e - b);
                    (void)r;
                }
            });
        for (auto& x : th) x.join();
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    std::printf("pieces: data node %d, pack threads %u on node %d, out %s: %7.1f GB/s\n", dataNode, T, packNode,
                g_pinned ? "pinned" : "malloc", n / best / 1e9);
    std::free(in);
    if (g_pinned) (void)hipHostFree(out);
    else std::free(out);
}

int main(int argc, char** argv) {
    const uint64_t n = (argc > 1 ? std::atoll(argv[1]) : 1024) << 20;
    std::vector<uint8_t> in(n), out(n / 4 + 64);
    std::mt19937_64 g(1);
    const uint8_t code[4] = {1, 2, 3, 5};
    for (uint64_t i = 0; i < n; i += 32) {
        uint64_t x = g();
        for (int j = 0; j < 32 && i + j < n; ++j) in[i + j] = code[(x >> (2 * j)) & 3];
    }
    std::memset(out.data(), 0, out.size());
    const bool has512 = __builtin_cpu_supports("avx512bw");
    std::printf("cpus %u, avx512bw %d, %llu MB\n", std::thread::hardware_concurrency(), has512 ? 1 : 0,
                (unsigned long long)(n >> 20));
    if (argc > 2) {
        g_pinned = argc > 3 && std::string(argv[3]) == "pinned";
        for (unsigned T : {8u, 16u})
            for (int dn : {0, 1})
                for (int pn : {0, 1, -1}) numaCase(n, dn, pn, T);
        return 0;
    }
    for (unsigned T : {1u, 4u, 8u, 16u}) {
        for (int v = 0; v < 4; ++v) {
            if (v >= 2 && !has512) continue;
            double best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                std::vector<std::thread> th;
                auto t0 = std::chrono::steady_clock::now();
                for (unsigned t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const uint64_t b = (n / T * t) & ~uint64_t(127), e = t + 1 == T ? n : (n / T * (t + 1)) & ~uint64_t(127);
                        volatile uint64_t r = v == 0 ? pack2<false>(in.data() + b, out.data() + b / 4, e - b)
                                            : v == 1 ? pack2<true>(in.data() + b, out.data() + b / 4, e - b)
                                            : v == 2 ? pack512<false>(in.data() + b, out.data() + b / 4, e - b)
                                                     : pack512<true>(in.data() + b, out.data() + b / 4, e - b);
                        (void)r;
                    });
                for (auto& x : th) x.join();
                best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
            static const char* names[] = {"avx2", "avx2+pf", "avx512", "avx512+pf"};
            std::printf("threads %2u %-10s %7.1f GB/s  %6.2f ms\n", T, names[v], n / best / 1e9, best * 1e3);
        }
    }
}
