// gather_bench.hip — ceiling of random 64-B line gathers on MI355X vs footprint.
// Each lane issues U independent random line reads per iteration (16 or 48 B
// of each 64-B line); reports lines/s. Footprints beyond the TLB reach show
// the translation cost the FM-index search pays on its Occ lines.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <int U, int W>
__global__ __launch_bounds__(256) void kGather(const uint4* __restrict__ buf, uint64_t nlines, uint32_t iters,
                                               uint64_t window, unsigned long long* sink) {
    const uint64_t gtid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t x = mix(gtid * 0x9E3779B97F4A7C15ull + 1);
    uint32_t acc = 0;
    // window: restrict a wave to a random window of `window` lines (0 = whole buffer)
    uint64_t base = 0, span = nlines;
    if (window) {
        uint64_t wv = mix(gtid / 64 + 7);
        span = window;
        base = (wv % (nlines / window)) * window;
    }
    for (uint32_t i = 0; i < iters; ++i) {
        uint4 v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x = mix(x + u + 1);
            const uint4* p = buf + (base + __umul64hi(x, span)) * 4;
#pragma unroll
            for (int w = 0; w < W; ++w) v[u][w] = p[w];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < W; ++w) acc ^= v[u][w].x ^ v[u][w].w;
    }
    if (acc == 0x9e3779b9u) atomicAdd(sink, 1ull);
}

template <int U, int W>
void run(const char* name, const uint4* buf, uint64_t nlines, uint64_t window, int blocksPerCU, int cus) {
    unsigned long long* sink;
    CK(hipMalloc(&sink, 8));
    const uint32_t iters = 64;
    const int blocks = cus * blocksPerCU;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((kGather<U, W>), dim3(blocks), dim3(256), 0, 0, buf, nlines, iters, window, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int reps = 3;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((kGather<U, W>), dim3(blocks), dim3(256), 0, 0, buf, nlines, iters, window, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double lines = (double)blocks * 256 * iters * U * reps;
    printf("%-34s footprint %7.2f GB window %9llu lines  U=%d W=%d blocks/CU=%d : %7.2f Glines/s = %7.1f GB/s (64B lines)\n",
           name, nlines * 64 / 1e9, (unsigned long long)window, U, W, blocksPerCU, lines / (ms / 1e3) / 1e9,
           lines * 64 / (ms / 1e3) / 1e9);
    CK(hipFree(sink));
}


// G lanes cooperate on one 64-B line: lane j of a group loads bytes
// [j*64/G, (j+1)*64/G). One wave instruction then touches 64/G distinct lines.
template <int U, int G>
__global__ __launch_bounds__(256) void kGroup(const uint8_t* __restrict__ buf, uint64_t nlines, uint32_t iters,
                                              unsigned long long* sink) {
    const uint64_t gtid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint32_t j = threadIdx.x % G;
    uint64_t x = mix((gtid / G) * 0x9E3779B97F4A7C15ull + 1);
    uint32_t acc = 0;
    constexpr int B = 64 / G;  // bytes per lane
    for (uint32_t i = 0; i < iters; ++i) {
        uint32_t v[U][B / 4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x = mix(x + u + 1);
            const uint8_t* p = buf + __umul64hi(x, nlines) * 64 + j * B;
            if constexpr (B == 16) { uint4 t = *reinterpret_cast<const uint4*>(p); v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w; }
            else if constexpr (B == 32) { uint4 t = *reinterpret_cast<const uint4*>(p); uint4 t2 = *reinterpret_cast<const uint4*>(p + 16);
                v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w; v[u][4] = t2.x; v[u][5] = t2.y; v[u][6] = t2.z; v[u][7] = t2.w; }
            else { uint2 t = *reinterpret_cast<const uint2*>(p); v[u][0] = t.x; v[u][1] = t.y; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < B / 4; ++w) acc ^= v[u][w];
    }
    if (acc == 0x9e3779b9u) atomicAdd(sink, 1ull);
}

template <int U, int G>
void runG(const char* name, const uint4* buf, uint64_t nlines, int blocksPerCU, int cus) {
    unsigned long long* sink;
    CK(hipMalloc(&sink, 8));
    const uint32_t iters = 64;
    const int blocks = cus * blocksPerCU;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((kGroup<U, G>), dim3(blocks), dim3(256), 0, 0, (const uint8_t*)buf, nlines, iters, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int reps = 3;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((kGroup<U, G>), dim3(blocks), dim3(256), 0, 0, (const uint8_t*)buf, nlines, iters, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double lines = (double)blocks * 256 / G * iters * U * reps;
    printf("%-34s footprint %7.2f GB  U=%d G=%d blocks/CU=%d : %7.2f Glines/s = %7.1f GB/s (64B lines)\n",
           name, nlines * 64 / 1e9, U, G, blocksPerCU, lines / (ms / 1e3) / 1e9, lines * 64 / (ms / 1e3) / 1e9);
    CK(hipFree(sink));
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const uint64_t maxBytes = 24ull << 30;
    uint4* buf;
    CK(hipMalloc(&buf, maxBytes));
    CK(hipMemset(buf, 1, maxBytes));
    const double sizesGB[] = {0.125, 6.75, 24.0};
    for (double gb : sizesGB) {
        const uint64_t nlines = (uint64_t)(gb * (1ull << 30)) / 64;
        run<4, 3>("lane/line 48B (3 loads)", buf, nlines, 0, 8, cus);
        runG<4, 2>("pair/line 32B/lane (2 loads)", buf, nlines, 8, cus);
        runG<4, 4>("quad/line 16B/lane (1 load)", buf, nlines, 8, cus);
        runG<8, 4>("quad/line U8", buf, nlines, 8, cus);
        runG<16, 4>("quad/line U16", buf, nlines, 8, cus);
        runG<4, 8>("oct/line 8B/lane (1 load)", buf, nlines, 8, cus);
        runG<8, 8>("oct/line U8", buf, nlines, 8, cus);
    }
    CK(hipFree(buf));
    return 0;
}
