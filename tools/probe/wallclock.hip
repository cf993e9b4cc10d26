#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
__global__ void k(unsigned long long* o) { o[0] = wall_clock64(); o[1] = clock64(); }
int main() {
  int khz = 0; hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  int ckhz = 0; hipDeviceGetAttribute(&ckhz, hipDeviceAttributeClockRate, 0);
  unsigned long long *d, h[2], h2[2]; hipMalloc(&d, 16);
  k<<<1,1>>>(d); hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now()-t0).count() < 0.5) {}
  k<<<1,1>>>(d); hipMemcpy(h2, d, 16, hipMemcpyDeviceToHost);
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now()-t0).count();
  printf("attr wallclock %d kHz, clock %d kHz; measured wall %.1f MHz, shader %.1f MHz\n", khz, ckhz, (h2[0]-h[0])/dt/1e6, (h2[1]-h[1])/dt/1e6);
}
