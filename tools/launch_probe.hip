// Fixed cost of a short dependent launch pair issued from an idle device (the driver's 20-step
// bench call: count kernel -> step kernel -> synchronise), by what precedes it on the host:
//   sync      the previous work synchronised (hipDeviceSynchronize), nothing recorded after it
//   event     + a hipEventRecord on the launch stream after the synchronisation (bench.py ev0)
//   sleepN    + N us of host sleep before the launches (the GPU idles that long)
//   stream    launches on the null stream / a created non-blocking stream
// Two kernels: a 2-us busy kernel (s_memrealtime spin on one block) and its dependent successor.
// Prints host wall time from the first launch to the return of the synchronisation (median of 200).
//   hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o tools/bin/launch_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
      std::exit(2);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void k_spin(unsigned long long ticks, int* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1;
}

using clk = std::chrono::steady_clock;

static double run(hipStream_t s, bool event, int sleep_us, int grid, int* d, hipEvent_t ev) {
  std::vector<double> v;
  for (int rep = 0; rep < 200; ++rep) {
    CK(hipDeviceSynchronize());
    if (event) CK(hipEventRecord(ev, s));
    if (event) CK(hipDeviceSynchronize());
    if (sleep_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    const auto t0 = clk::now();
    hipLaunchKernelGGL(k_spin, dim3(grid), dim3(256), 0, s, 200ull, d);  // 2 us at 100 MHz
    hipLaunchKernelGGL(k_spin, dim3(grid), dim3(256), 0, s, 200ull, d);
    CK(hipStreamSynchronize(s));
    v.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  int* d = nullptr;
  CK(hipMalloc(&d, 64));
  hipStream_t mine;
  CK(hipStreamCreateWithFlags(&mine, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreate(&ev));
  for (int grid : {1, 2048}) {
    for (int on_null : {1, 0}) {
      hipStream_t s = on_null ? (hipStream_t)0 : mine;
      for (int event : {0, 1}) {
        for (int sl : {0, 100, 1000}) {
          const double us = run(s, event, sl, grid, d, ev);
          std::printf("grid %4d stream %-7s event %d sleep %4d us: launch pair + sync %.1f us (2 x 2 us of kernel)\n",
                      grid, on_null ? "null" : "created", event, sl, us);
        }
      }
    }
  }
  return 0;
}
