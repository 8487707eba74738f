// mdr_actor.hip — MA-PPO actor forward fused with the observation.
//
// Reference: Actor.forward (server/app/core/agents/trainables/network.py:29-33) =
// softmax(fc2(relu(fc1(relu(fc0(x)))))) over the norm_state_dict vector (server/app/utils/norm.py:
// 178-218), sampled per agent with Categorical (server/app/core/agents/trainables/mappo.py:83-97).
// The reference runs N batch-1 forwards on the CPU; here one persistent launch builds each house's
// observation row in LDS (never written to HBM unless asked), runs the two hidden layers as MFMA
// tiles (houses on the 32 columns of v_mfma_f32_32x32x16_bf16, neurons on the rows), the output
// layer + softmax + sampling on the VALU, and writes action (u8) and the chosen action's
// probability (f32).  Optionally it also counts the ON houses per capacity class the new actions
// produce (the next k_step's cluster power), so a policy tick + env tick is two launches.
//
// Precision (mdr_actor_spec.precision):
//   MDR_PREC_BF16X3 — every fp32 operand x is split x = hi + lo (hi = bf16(x), lo = bf16(x - hi))
//                     and a·b ≈ ah·bh + ah·bl + al·bh, accumulated in fp32: ~1e-5 relative to the
//                     fp32 reference (bf16 alone: ~4e-3).
//   MDR_PREC_BF16   — one bf16 product per term.
// Bias adds, ReLU, the output layer, softmax and sampling are fp32.
//
// Fragment maps (gfx950, 32x32x16 bf16; lane l, r = l & 31, h = l >> 5, element j = 0..7):
//   A[row r][k = 8h + j], B[k = 8h + j][col r], C/D reg g: col r, row (g & 3) + 8 (g >> 2) + 4h.
// Layer 2 takes layer 1's accumulator registers 8s .. 8s+7 of row block kb directly as its B
// fragment for k-step q = 2 kb + s: element j is hidden row 16q + 8 (j >> 2) + 4h + (j & 3); the
// packed W2 fragments use that same k order (k_actor_pack), so no lane movement is needed.
#include "mdr_actor.h"
#include "mdr_obs_dev.h"

namespace mdr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// --------------------------------------------------------------------------------------- pack
// One thread per (fragment, lane): 8 weights -> bf16 hi (and lo) in fragment order.
__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (__bf16)v[j];
    lo[j] = (__bf16)(v[j] - (float)hi[j]);
  }
}

__global__ void k_actor_pack(ActorDims d, const float* __restrict__ w1, const float* __restrict__ b1,
                             const float* __restrict__ w2, const float* __restrict__ b2,
                             const float* __restrict__ w3, const float* __restrict__ b3,
                             unsigned char* __restrict__ out) {
  const int nf1 = kActorMB * d.ks1, nf2 = kActorMB * d.ks2;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = g & 63, f = g >> 6;
  const int r = lane & 31, h = lane >> 5;
  float v[8];
  bf16x8 hi, lo;
  if (f < nf1) {  // W1 [H1][n_in], fragment (mb, ks)
    const int mb = f / d.ks1, ks = f % d.ks1;
    const int row = 32 * mb + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * ks + 8 * h + j;
      v[j] = (row < d.h1 && k < d.n_in) ? w1[row * d.n_in + k] : 0.f;
    }
    split8(v, hi, lo);
    reinterpret_cast<bf16x8*>(out + d.off_w1)[(2 * f) * 64 + lane] = hi;
    reinterpret_cast<bf16x8*>(out + d.off_w1)[(2 * f + 1) * 64 + lane] = lo;
  } else if (f < nf1 + nf2) {  // W2 [H2][H1], fragment (mb, q) in the accumulator k order
    const int f2 = f - nf1;
    const int mb = f2 / d.ks2, q = f2 % d.ks2;
    const int row = 32 * mb + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * q + 8 * (j >> 2) + 4 * h + (j & 3);
      v[j] = (row < d.h2 && k < d.h1) ? w2[row * d.h1 + k] : 0.f;
    }
    split8(v, hi, lo);
    reinterpret_cast<bf16x8*>(out + d.off_w2)[(2 * f2) * 64 + lane] = hi;
    reinterpret_cast<bf16x8*>(out + d.off_w2)[(2 * f2 + 1) * 64 + lane] = lo;
  } else if (f == nf1 + nf2) {  // fp32 tail: b1, b2 [128], W3 [n_act][128], b3 [n_act]
    float* t = reinterpret_cast<float*>(out + d.off_tail);
    for (int i = lane; i < kActorRows; i += 64) {
      t[i] = i < d.h1 ? b1[i] : 0.f;
      t[kActorRows + i] = i < d.h2 ? b2[i] : 0.f;
      for (int a = 0; a < d.n_act; ++a) t[2 * kActorRows + a * kActorRows + i] = i < d.h2 ? w3[a * d.h2 + i] : 0.f;
    }
    if (lane < d.n_act) t[(2 + d.n_act) * kActorRows + lane] = b3[lane];
  }
}

// --------------------------------------------------------------------------------------- forward
__device__ __forceinline__ bf16x8 lds_frag(const unsigned char* base, int frag, int lane) {
  return reinterpret_cast<const bf16x8*>(base)[frag * 64 + lane];
}

__device__ __forceinline__ float philox_u01f(uint64_t seed, uint64_t gid, uint64_t tick) {
  const u32x4 c = philox4x32_10(u32x4{(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)tick,
                                      (uint32_t)(tick >> 32) ^ 0xAC7u},
                                (uint32_t)seed ^ 0x3C6EF372u, (uint32_t)(seed >> 32));
  return (float)(c.x >> 8) * (1.0f / 16777216.0f);  // [0, 1), 24 bits
}

template <int PREC>
__global__ void __launch_bounds__(512) k_actor(KParams p, ObsArgs o, ActorDims d, const double* p_dev,
                                               const unsigned char* __restrict__ wpack, ActorOut out,
                                               uint64_t tick0, const TickArgs* tkp) {
  const uint64_t tick = tkp ? tkp->tick : tick0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nthr = blockDim.x, nw = nthr >> 6;
  const int HB = 32 * nw;  // houses per block iteration
  const int r = lane & 31, h = lane >> 5;
  const int F = o.n_feat, FS = d.fs;

  // LDS carve-up (byte offsets computed on the host, mdr_actor_lds)
  unsigned char* s_w1 = smem;
  unsigned char* s_w2 = smem + d.off_w2;
  const float* s_tail = reinterpret_cast<const float*>(smem + d.off_tail);
  float* s_obs = reinterpret_cast<float*>(smem + d.lds_obs);     // [HB][FS] + 16 ks1
  float* s_msg = reinterpret_cast<float*>(smem + d.lds_msg);     // [lo + HB + hi][M]
  uint32_t* s_hw = reinterpret_cast<uint32_t*>(smem + d.lds_hw); // [HB] hvac words
  unsigned* s_hist = reinterpret_cast<unsigned*>(smem + d.lds_hist);

  // weights -> LDS once per block (PREC 1 skips the lo fragments)
  {
    const uint4* src = reinterpret_cast<const uint4*>(wpack);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = d.off_end / 16;
    for (int q = tid; q < n16; q += nthr) {
      if (PREC == 1 && q < d.off_tail / 16) {
        const int frag = q / 64;  // 1-KB fragments: even = hi, odd = lo
        if (frag & 1) continue;
      }
      dst[q] = src[q];
    }
    for (int q = tid; q < HB * FS + 16 * d.ks1; q += nthr) s_obs[q] = 0.f;  // + the k-padding overrun
    if (tid < MDR_MAX_CAP) s_hist[tid] = 0u;
  }
  const double P = p_dev ? *p_dev : o.p;
  if (o.sc_dev) { o.s = o.sc_dev[0]; o.solar = o.sc_dev[1]; o.t_od = o.sc_dev[2]; }
  const float* b1 = s_tail;
  const float* b2 = s_tail + kActorRows;
  const float* w3 = s_tail + 2 * kActorRows;
  const float* b3 = s_tail + (2 + d.n_act) * kActorRows;

  const int64_t n = p.n;
  const int64_t ntile = (n + HB - 1) / HB;
  for (int64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const int64_t b0 = tile * HB;
    const int nb = (int)min((int64_t)HB, n - b0);
    __syncthreads();  // previous iteration done with s_obs / s_msg (and the initial fill visible)
    obs_stage_ring(p, o, b0, nb, s_msg, tid, nthr);
    __syncthreads();
    if (tid < nb) {
      float* row = s_obs + tid * FS;
      s_hw[tid] = obs_build_row(p, o, P, b0 + tid, tid, s_msg, row);
      for (int f = F; f < FS; ++f) row[f] = 0.f;
    }
    __syncthreads();
    if (out.obs) {  // optional obs[b0 .. b0 + nb) rows to HBM (training buffers)
      const int64_t nflt = (int64_t)nb * F;
      float* dst = out.obs + b0 * F;
      for (int64_t q = tid; q < nflt; q += nthr) {
        const int rr = (int)(q / F);
        dst[q] = s_obs[rr * FS + (int)(q - (int64_t)rr * F)];
      }
    }

    // ---- layer 1: acc1[mb] = b1 + W1 · X  (X^T columns = this wave's 32 houses)
    const float* xrow = s_obs + (32 * wv + r) * FS + 8 * h;
    f32x16 acc1[kActorMB];
#pragma unroll
    for (int mb = 0; mb < kActorMB; ++mb)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc1[mb][g] = b1[32 * mb + (g & 3) + 8 * (g >> 2) + 4 * h];
    for (int ks = 0; ks < d.ks1; ++ks) {
      const float4 x0 = *reinterpret_cast<const float4*>(xrow + 16 * ks);
      const float4 x1 = *reinterpret_cast<const float4*>(xrow + 16 * ks + 4);
      const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 xh, xl;
      split8(xv, xh, xl);
      bf16x8 ah[kActorMB], al[kActorMB];
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb) {
        const int f = mb * d.ks1 + ks;
        ah[mb] = lds_frag(s_w1, 2 * f, lane);
        if (PREC == 3) al[mb] = lds_frag(s_w1, 2 * f + 1, lane);
      }
      if (PREC == 3) {
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mb], xh, acc1[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], xl, acc1[mb], 0, 0, 0);
      }
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], xh, acc1[mb], 0, 0, 0);
    }

    // ---- ReLU + split: layer 1's accumulators become layer 2's B fragments in place
    bf16x8 hh[2 * kActorMB], hl[2 * kActorMB];
#pragma unroll
    for (int q = 0; q < 2 * kActorMB; ++q) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(acc1[q >> 1][8 * (q & 1) + j], 0.f);
      split8(v, hh[q], hl[q]);
    }

    // ---- layer 2: acc2[mb] = b2 + W2 · relu(H1)
    f32x16 acc2[kActorMB];
#pragma unroll
    for (int mb = 0; mb < kActorMB; ++mb)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc2[mb][g] = b2[32 * mb + (g & 3) + 8 * (g >> 2) + 4 * h];
#pragma unroll
    for (int q = 0; q < 2 * kActorMB; ++q) {
      if (q >= d.ks2) break;
      bf16x8 ah[kActorMB], al[kActorMB];
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb) {
        const int f = mb * d.ks2 + q;
        ah[mb] = lds_frag(s_w2, 2 * f, lane);
        if (PREC == 3) al[mb] = lds_frag(s_w2, 2 * f + 1, lane);
      }
      if (PREC == 3) {
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mb], hh[q], acc2[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], hl[q], acc2[mb], 0, 0, 0);
      }
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], hh[q], acc2[mb], 0, 0, 0);
    }

    // ---- output layer (fp32 VALU): this lane's 64 hidden rows, then the partner half's
    float z[kActorMaxAct];
#pragma unroll
    for (int a = 0; a < kActorMaxAct; ++a) z[a] = 0.f;
#pragma unroll
    for (int mb = 0; mb < kActorMB; ++mb)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int row = 32 * mb + (g & 3) + 8 * (g >> 2) + 4 * h;
        const float x = fmaxf(acc2[mb][g], 0.f);
#pragma unroll
        for (int a = 0; a < kActorMaxAct; ++a)
          if (a < d.n_act) z[a] += w3[a * kActorRows + row] * x;
      }
#pragma unroll
    for (int a = 0; a < kActorMaxAct; ++a)
      if (a < d.n_act) z[a] = z[a] + __shfl_xor(z[a], 32) + b3[a];

    // ---- softmax (fp32, max-subtracted like torch) + Categorical sample
    float zmax = z[0];
#pragma unroll
    for (int a = 1; a < kActorMaxAct; ++a)
      if (a < d.n_act) zmax = fmaxf(zmax, z[a]);
    float e[kActorMaxAct], se = 0.f;
#pragma unroll
    for (int a = 0; a < kActorMaxAct; ++a)
      if (a < d.n_act) { e[a] = expf(z[a] - zmax); se += e[a]; }
    const int hl_ = 32 * wv + r;  // house within the block tile
    const bool valid = hl_ < nb;
    const int64_t i = b0 + hl_;
    const float u = philox_u01f(p.seed, (uint64_t)(p.goff + i), tick);
    // Categorical(probs).sample(): first action whose cumulative probability exceeds u
    float pr[kActorMaxAct];
    int act = d.n_act - 1;
    float cum = 0.f;
    bool found = false;
#pragma unroll
    for (int a = 0; a < kActorMaxAct; ++a)
      if (a < d.n_act) {
        pr[a] = e[a] / se;
        if (out.probs && valid && h == 0) out.probs[i * d.n_act + a] = pr[a];
        if (a < d.n_act - 1 && !found) {
          cum += pr[a];
          if (u < cum) { act = a; found = true; }
        }
      }
    float pa = 0.f;
#pragma unroll
    for (int a = 0; a < kActorMaxAct; ++a)
      if (a == act) pa = pr[a];
    if (valid && h == 0) {
      if (out.action) out.action[i] = (uint8_t)act;
      if (out.prob) out.prob[i] = pa;
    }
    if (out.count_next) {
      // the ON houses the new actions produce (hvac.py:43-64 on action != 0), per capacity class
      const bool on1 = valid && h == 0 && hv_on(hvac_fsm(s_hw[hl_], act != 0, p.dt, p.L));
      const int cls = valid ? p.cap_idx[i] : 0;
      for (int k = 0; k < p.n_cap; ++k) {
        const unsigned long long m = __ballot(on1 && cls == k);
        if (lane == 0 && m) atomicAdd(&s_hist[k], (unsigned)__popcll(m));
      }
    }
  }
  if (out.count_next) {
    __syncthreads();
    if (tid < p.n_cap && s_hist[tid])
      atomicAdd(&out.count_next[(blockIdx.x % kCountShards) * p.n_cap + tid], (unsigned long long)s_hist[tid]);
  }
}

template __global__ void k_actor<1>(KParams, ObsArgs, ActorDims, const double*, const unsigned char*,
                                    ActorOut, uint64_t, const TickArgs*);
template __global__ void k_actor<3>(KParams, ObsArgs, ActorDims, const double*, const unsigned char*,
                                    ActorOut, uint64_t, const TickArgs*);

}  // namespace mdr
