// Probe: where does one global_load_lds wave-instruction of size 4 / 12 / 16
// put each lane's bytes in LDS (gfx950)? Source words are tagged
// (lane << 8 | word); a few lanes are masked off.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(1))) void* glb_ptr;

#define KERNEL(NAME, SIZE)                                                            \
__global__ void NAME(const uint32_t* src, uint32_t* out) {                            \
    __shared__ uint32_t lds[64 * 8];                                                  \
    const uint32_t t = threadIdx.x;                                                   \
    for (uint32_t i = t; i < 64 * 8; i += 64) lds[i] = 0xFFFFFFFFu;                   \
    __syncthreads();                                                                  \
    if (t != 1) __builtin_amdgcn_global_load_lds((glb_ptr)(src + 4 * t), (lds_ptr)lds, SIZE, 0, 0); \
    __builtin_amdgcn_s_waitcnt(0);                                                    \
    __syncthreads();                                                                  \
    for (uint32_t i = t; i < 64 * 8; i += 64) out[i] = lds[i];                        \
}
KERNEL(k4, 4)
KERNEL(k12, 12)
KERNEL(k16, 16)
template <int SIZE>
__global__ void k_unused(const uint32_t* src, uint32_t* out) {
    __shared__ uint32_t lds[64 * 8];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 64 * 8; i += 64) lds[i] = 0xFFFFFFFFu;
    __syncthreads();
    (void)src;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (uint32_t i = t; i < 64 * 8; i += 64) out[i] = lds[i];
}

int main() {
    uint32_t h[64 * 4];
    for (int l = 0; l < 64; ++l)
        for (int w = 0; w < 4; ++w) h[l * 4 + w] = (uint32_t)(l << 8 | w);
    uint32_t *src, *out;
    hipMalloc(&src, sizeof(h));
    hipMalloc(&out, 64 * 8 * 4);
    hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
    uint32_t o[64 * 8];
    auto show = [&](const char* name) {
        hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
        printf("%s:", name);
        for (int i = 0; i < 20; ++i) printf(" %x", o[i]);
        printf(" ... [255..260]:");
        for (int i = 255; i < 261; ++i) printf(" %x", o[i]);
        printf("\n");
    };
    hipLaunchKernelGGL(k4, dim3(1), dim3(64), 0, 0, src, out); show("size4");
    hipLaunchKernelGGL(k12, dim3(1), dim3(64), 0, 0, src, out); show("size12");
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, src, out); show("size16");
    return 0;
}
