// Cycles per MFMA on one SIMD for the bf16 forms the actor kernel can use:
// v_mfma_f32_16x16x32_bf16 (K = 32), v_mfma_f32_16x16x16_bf16 (K = 16) and
// v_mfma_f32_32x32x16_bf16 (twice the work of 16x16x32 per instruction), back to back on
// NACC independent accumulators, one wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/bin/mfma_probe && tools/bin/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// FORM 0: 16x16x32, 1: 16x16x16, 2: 32x32x16
template <int FORM, int NACC>
__global__ void probe(float* out, long long* cyc, int iters) {
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int j = 0; j < 8; ++j) { a8[j] = (__bf16)(threadIdx.x * 0.001f + j); b8[j] = (__bf16)(j * 0.5f); }
  for (int j = 0; j < 4; ++j) { a4[j] = a8[j]; b4[j] = b8[j]; }
  f32x4 c[NACC] = {};
  f32x16 d[NACC] = {};
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < NACC; ++u) {
      if constexpr (FORM == 0) c[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c[u], 0, 0, 0);
      else if constexpr (FORM == 1) c[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c[u], 0, 0, 0);
      else d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d[u], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int u = 0; u < NACC; ++u) {
    for (int j = 0; j < 4; ++j) s += c[u][j];
    for (int j = 0; j < 16; ++j) s += d[u][j];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int FORM, int NACC>
void run(float* out, long long* cyc, const char* name, double flops) {
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((probe<FORM, NACC>), dim3(256), dim3(64), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
  }
  long long h = 0;
  hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const double c = (double)h / ((double)NACC * iters);
  printf("%-14s %d acc: %6.2f cycles per MFMA, %7.1f flops per cycle per SIMD\n", name, NACC, c, flops / c);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 64 * sizeof(float));
  hipMalloc(&cyc, sizeof(long long));
  run<0, 4>(out, cyc, "16x16x32 bf16", 2.0 * 16 * 16 * 32);
  run<0, 8>(out, cyc, "16x16x32 bf16", 2.0 * 16 * 16 * 32);
  run<1, 4>(out, cyc, "16x16x16 bf16", 2.0 * 16 * 16 * 16);
  run<2, 2>(out, cyc, "32x32x16 bf16", 2.0 * 32 * 32 * 16);
  run<2, 4>(out, cyc, "32x32x16 bf16", 2.0 * 32 * 32 * 16);
  return 0;
}
