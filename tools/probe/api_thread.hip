// HIP API cost on the main thread against a helper thread (r6 thread probe,
// DESIGN.md §9): empty-kernel launches, event records/queries and stream
// waits, timed per call. Build: hipcc --offload-arch=gfx950 -O2 api_thread.hip -o api_thread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

__global__ void kEmpty(int* p) {
    if (threadIdx.x == 1024) *p = 0;
}

__global__ void kSpin(long long cycles) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}

// does a cross-stream wait on a pending event hold the calling thread?
static void waitHolds(const char* who, hipStream_t a, hipStream_t b, hipEvent_t e) {
    hipLaunchKernelGGL(kSpin, dim3(1), dim3(64), 0, a, 200000LL);  // ~2 ms at 100 MHz
    (void)hipEventRecord(e, a);
    auto t0 = std::chrono::steady_clock::now();
    (void)hipStreamWaitEvent(b, e, 0);
    hipLaunchKernelGGL(kSpin, dim3(1), dim3(64), 0, b, 1000LL);
    auto t1 = std::chrono::steady_clock::now();
    (void)hipDeviceSynchronize();
    auto t2 = std::chrono::steady_clock::now();
    std::printf("%-7s wait+launch behind a 2-ms kernel returned after %.1f us (all done at %.1f us)\n", who,
                std::chrono::duration<double, std::micro>(t1 - t0).count(),
                std::chrono::duration<double, std::micro>(t2 - t0).count());
}

static void run(const char* who, hipStream_t a, hipStream_t b, hipEvent_t e, int* d) {
    constexpr int kN = 20000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < kN; ++i) hipLaunchKernelGGL(kEmpty, dim3(1), dim3(64), 0, a, d);
    auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(a);
    auto t2 = std::chrono::steady_clock::now();
    for (int i = 0; i < kN; ++i) {
        (void)hipEventRecord(e, a);
        (void)hipStreamWaitEvent(b, e, 0);
    }
    auto t3 = std::chrono::steady_clock::now();
    for (int i = 0; i < kN; ++i) (void)hipEventQuery(e);
    auto t4 = std::chrono::steady_clock::now();
    (void)hipDeviceSynchronize();
    auto us = [](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count() / kN; };
    std::printf("%-7s launch %.2f us (drain %.2f us/kernel), record+wait %.2f us, query %.2f us\n", who, us(t0, t1),
                us(t1, t2), us(t2, t3), us(t3, t4));
}

int main() {
    (void)hipSetDevice(0);
    hipStream_t a, b;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    hipEvent_t e;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    int* d = nullptr;
    (void)hipMalloc(&d, 4);
    for (int r = 0; r < 2; ++r) {
        run("main", a, b, e, d);
        waitHolds("main", a, b, e);
        std::thread([&] {
            (void)hipSetDevice(0);
            run("helper", a, b, e, d);
            waitHolds("helper", a, b, e);
        }).join();
        // streams made on the helper, used from main and from a helper
        hipStream_t c = nullptr, f = nullptr;
        std::thread([&] {
            (void)hipSetDevice(0);
            (void)hipStreamCreateWithFlags(&c, hipStreamNonBlocking);
            (void)hipStreamCreateWithFlags(&f, hipStreamNonBlocking);
        }).join();
        waitHolds("main(h)", c, f, e);
        std::thread([&] {
            (void)hipSetDevice(0);
            waitHolds("help(h)", c, f, e);
        }).join();
    }
    return 0;
}
