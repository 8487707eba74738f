// Does a SIMD overlap one wave's MFMAs with another wave's VALU work?  One block of 8 waves per CU
// (waves w and w + 4 share a SIMD): waves 0-3 run a chain of v_mfma_f32_16x16x32_bf16 on 4
// independent accumulators, waves 4-7 run fp32 FMAs (8 independent chains) or fp64 FMAs; each
// alone, then both.  Prints kernel time by HIP events: both ~ max(alone) means the matrix pipe and
// the VALU overlap across waves; both ~ sum means they do not.  Also the same mixes inside ONE wave
// (MFMAs interleaved with independent VALU ops).
//   hipcc --offload-arch=gfx950 -O3 tools/overlap_probe.hip -o tools/bin/overlap_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// MODE bit 0: waves 0-3 run MFMAs; bit 1: waves 4-7 run VALU; bit 2: fp64 VALU instead of fp32;
// bit 3: one wave does both (waves 0-3 interleave VALU ops between their MFMAs, waves 4-7 idle);
// bit 4: waves 4-7 run MFMAs too (two MFMA waves per SIMD).  The MFMA operands live in VGPRs (no
// VALU write of an MFMA source inside the loop).  cyc: clock64 ticks of wave 0 of block 0
template <int MODE>
__global__ void __launch_bounds__(512) probe(float* out, int iters, int vper, long long* cyc) {
  const int wv = threadIdx.x >> 6;
  bf16x8 a8, b8;
  for (int j = 0; j < 8; ++j) {
    a8[j] = (__bf16)(threadIdx.x * 0.001f + j);
    b8[j] = (__bf16)(j * 0.5f + threadIdx.x * 0.002f);
  }
  f32x4 c[4] = {};
  float v[8];
  double w[8];
  uint32_t x[8];
  for (int j = 0; j < 8; ++j) { v[j] = threadIdx.x * 1e-3f + j; w[j] = v[j]; x[j] = threadIdx.x * 977u + j; }
  const float fa = 0.999f + threadIdx.x * 1e-9f, fb = 1e-3f;
  const double da = 0.999 + threadIdx.x * 1e-12, db = 1e-3;
  const bool mf = ((MODE & 1) && wv < 4) || ((MODE & 16) && wv >= 4);
  const bool va = ((MODE & 2) && wv >= 4) || ((MODE & 8) && wv < 4);
  const long long t0 = clock64();
  auto valu = [&]() {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MODE & 32) x[j] = (x[j] ^ (x[j] << 5)) + 0x9E3779B9u;  // 32-bit integer ops (3 per element)
      else if (MODE & 4) w[j] = __builtin_fma(w[j], da, db);
      else v[j] = __builtin_fmaf(v[j], fa, fb);
    }
  };
  if (mf && va) {  // one wave: VALU ops between the MFMAs
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 4; ++u) c[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c[u], 0, 0, 0);
      for (int r = 0; r < vper; ++r) valu();
    }
  } else if (mf) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 4; ++u) c[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c[u], 0, 0, 0);
    }
  } else if (va) {
    for (int i = 0; i < iters * vper; ++i) valu();
  }
  const long long t1 = clock64();
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
  float s = 0.f;
  for (int u = 0; u < 4; ++u) s += c[u][0] + c[u][1] + c[u][2] + c[u][3];
  for (int j = 0; j < 8; ++j) s += v[j] + (float)w[j] + (float)x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one wave per SIMD (waves 0-3 of a 512-thread block), NACC independent accumulators, DEP
// dependent MFMAs per accumulator in a row (the actor's split products: DEP = 3) before the next
template <int NACC, int DEP>
__global__ void __launch_bounds__(512) chains(float* out, int n_mfma, long long* cyc) {
  const int wv = threadIdx.x >> 6;
  bf16x8 a8, b8;
  for (int j = 0; j < 8; ++j) { a8[j] = (__bf16)(threadIdx.x * 0.001f + j); b8[j] = (__bf16)(j * 0.5f); }
  f32x4 c[NACC] = {};
  const long long t0 = clock64();
  if (wv < 4) {
    for (int i = 0; i < n_mfma / (NACC * DEP); ++i) {
#pragma unroll
      for (int u = 0; u < NACC; ++u)
#pragma unroll
        for (int k = 0; k < DEP; ++k) c[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c[u], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
  float s = 0.f;
  for (int u = 0; u < NACC; ++u) s += c[u][0] + c[u][1] + c[u][2] + c[u][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

long long* g_cyc;
long long last_cyc() {
  long long h = 0;
  hipMemcpy(&h, g_cyc, sizeof(h), hipMemcpyDeviceToHost);
  return h;
}
template <int MODE>
float run(float* out, int iters, int vper) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, out, iters, vper, g_cyc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    if (rep > 0 && ms < best) best = ms;
  }
  return best * 1e3f;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * sizeof(float));
  hipMalloc(&g_cyc, sizeof(long long));
  const int iters = 2048;
  {
    const float m1 = run<1>(out, iters, 1);
    const long long c1 = last_cyc();
    const float m2 = run<17>(out, iters, 1);
    const long long c2 = last_cyc();
    printf("MFMA: one wave per SIMD %.1f us (%lld clock64 ticks = %.1f per MFMA, %.2f GHz by ticks/time); two waves "
           "per SIMD (twice the MFMAs) %.1f us (%lld ticks)\n", m1, c1, c1 / (4.0 * iters), c1 / (m1 * 1e3), m2, c2);
  }
  {
    const int n = 8192 * 3;
    auto one = [&](auto kern, const char* name) {
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, n, g_cyc);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, n, g_cyc);
      hipDeviceSynchronize();
      printf("one wave, %-40s %.1f clock64 ticks per MFMA\n", name, last_cyc() / (double)n);
    };
    one(chains<1, 1>, "1 accumulator");
    one(chains<2, 1>, "2 accumulators");
    one(chains<4, 1>, "4 accumulators");
    one(chains<8, 1>, "8 accumulators");
    one(chains<2, 3>, "2 accumulators x 3 dependent (actor now)");
    one(chains<4, 3>, "4 accumulators x 3 dependent");
    one(chains<6, 3>, "6 accumulators x 3 dependent");
  }
  // vper rounds of 8 FMAs per iteration: 4 MFMAs = 64 matrix cycles per iteration
  for (int vper : {1, 2, 4}) {
    const float m = run<1>(out, iters, vper);
    const float f = run<2>(out, iters, vper), mf = run<3>(out, iters, vper), one = run<9>(out, iters, vper);
    const float d = run<6>(out, iters, vper), md = run<7>(out, iters, vper), oned = run<13>(out, iters, vper);
    const float q = run<34>(out, iters, vper), mq = run<35>(out, iters, vper), oneq = run<41>(out, iters, vper);
    printf("VALU %2d x 8 ops per 4 MFMAs | MFMA alone %7.1f us | fp32 (packed): alone %7.1f  both waves %7.1f  one wave "
           "%7.1f | fp64: alone %7.1f  both waves %7.1f  one wave %7.1f | int32 (x3): alone %7.1f  both waves %7.1f  "
           "one wave %7.1f\n",
           vper, m, f, mf, one, d, md, oned, q, mq, oneq);
  }
  return 0;
}
