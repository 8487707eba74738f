// Cycles per MFMA on one SIMD for the bf16 16x16 forms the actor kernel can use:
// v_mfma_f32_16x16x32_bf16 (K = 32) and v_mfma_f32_16x16x16_bf16 (K = 16), back to back on
// independent accumulators, one wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ void probe(float* out, long long* cyc, int iters) {
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int j = 0; j < 8; ++j) { a8[j] = (__bf16)(threadIdx.x * 0.001f + j); b8[j] = (__bf16)(j * 0.5f); }
  for (int j = 0; j < 4; ++j) { a4[j] = a8[j]; b4[j] = b8[j]; }
  f32x4 c[4] = {};
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (K == 32) c[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c[u], 0, 0, 0);
      else c[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c[u], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int u = 0; u < 4; ++u) s += c[u][0] + c[u][1] + c[u][2] + c[u][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 64 * sizeof(float));
  hipMalloc(&cyc, sizeof(long long));
  const int iters = 4096;
  for (int k = 0; k < 2; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      if (k == 0) hipLaunchKernelGGL(probe<32>, dim3(256), dim3(64), 0, 0, out, cyc, iters);
      else hipLaunchKernelGGL(probe<16>, dim3(256), dim3(64), 0, 0, out, cyc, iters);
      hipDeviceSynchronize();
    }
    long long h = 0;
    hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("16x16x%d bf16: %.2f cycles per MFMA (one wave per SIMD, 4 independent accumulators)\n", k == 0 ? 32 : 16,
           (double)h / (4.0 * iters));
  }
  return 0;
}
