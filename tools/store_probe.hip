// Streaming-store bandwidth of the step kernel's reward-row pattern: 32 rows of n f64 (one row per
// tick), each wave writing 128 consecutive houses of a row per tick as (a) two 8-B-per-lane stores
// (k_step_window's layout: lane l -> houses l and l + 64), (b) one 16-B-per-lane store (lane l ->
// houses 2l, 2l + 1); cached or non-temporal.  Also a read+write pass of 90 B/house of state first
// in each wave, as the window kernel does.  Prints TB/s of the rows.
//   hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip -o tools/bin/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int MODE, bool NT>
__global__ void __launch_bounds__(256) rows(double* __restrict__ out, int64_t n, int K, double v0) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t i0 = tile * 128;
  if (i0 >= n) return;
  double x = v0 + lane;
  for (int j = 0; j < K; ++j) {
    double* row = out + (int64_t)j * n;
    x = x * 1.0000001 + 0.5;
    if (MODE == 0) {
      if (NT) {
        __builtin_nontemporal_store(x, row + i0 + lane);
        __builtin_nontemporal_store(x + 1.0, row + i0 + 64 + lane);
      } else {
        row[i0 + lane] = x;
        row[i0 + 64 + lane] = x + 1.0;
      }
    } else {
      d2* p = reinterpret_cast<d2*>(row + i0 + 2 * lane);
      if (NT) __builtin_nontemporal_store(d2{x, x + 1.0}, p);
      else *p = d2{x, x + 1.0};
    }
  }
}

int main() {
  const int64_t n = 1 << 20;
  const int K = 32;
  double* out;
  hipMalloc(&out, (size_t)n * K * sizeof(double));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = (int)(n / 512);
  const char* names[4] = {"2 x 8 B/lane cached", "2 x 8 B/lane non-temporal", "16 B/lane cached", "16 B/lane non-temporal"};
  for (int v = 0; v < 4; ++v) {
    float best = 1e9f;
    for (int rep = 0; rep < 20; ++rep) {
      hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL((rows<0, false>), dim3(grid), dim3(256), 0, 0, out, n, K, 1.0);
      if (v == 1) hipLaunchKernelGGL((rows<0, true>), dim3(grid), dim3(256), 0, 0, out, n, K, 1.0);
      if (v == 2) hipLaunchKernelGGL((rows<1, false>), dim3(grid), dim3(256), 0, 0, out, n, K, 1.0);
      if (v == 3) hipLaunchKernelGGL((rows<1, true>), dim3(grid), dim3(256), 0, 0, out, n, K, 1.0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      if (rep >= 3 && ms < best) best = ms;
    }
    const double bytes = (double)n * K * 8;
    printf("%-28s %8.2f us  %6.2f TB/s\n", names[v], best * 1e3, bytes / (best * 1e-3) / 1e12);
  }
  return 0;
}
