// mdr_actor.hip — MA-PPO actor forward fused with the observation.
//
// Reference: Actor.forward (server/app/core/agents/trainables/network.py:29-33) =
// softmax(fc2(relu(fc1(relu(fc0(x)))))) over the norm_state_dict vector (server/app/utils/norm.py:
// 178-218), sampled per agent with Categorical (server/app/core/agents/trainables/mappo.py:83-97).
// The reference runs N batch-1 forwards on the CPU; here one persistent launch builds each house's
// observation on chip (never written to HBM unless asked), runs the two hidden layers as MFMA tiles
// (v_mfma_f32_16x16x32_bf16: neurons on the 16 rows of a row block, houses on the 16 columns; a
// wave's tile is 32 houses = two column blocks sharing every weight fragment it reads from LDS),
// the 2-wide output layer + softmax + sampling on the VALU, and writes action (u8) and the chosen
// action's probability (f32).  Optionally it also counts the ON houses per capacity class the new
// actions produce (the next k_step's cluster power), so a policy tick + env tick is two launches.
//
// Precision (mdr_actor_spec.precision):
//   MDR_PREC_BF16X3 — every fp32 operand x is split x = hi + lo (hi = bf16(x), lo = bf16(x - hi))
//                     and a·b ≈ ah·bh + ah·bl + al·bh, accumulated in fp32: ~1e-5 relative to the
//                     fp32 reference (bf16 alone: ~4e-3).
//   MDR_PREC_FP32   — fp32-faithful.  Default form (kernel PREC 4): an fp16 hi/lo split on
//                     v_mfma_f32_16x16x32_f16 (the bf16 rate): x = hi + lo with hi = fp16(x), lo =
//                     fp16(x - hi) — 11 + 11 significand bits against bf16's 8 + 8 — and a·b ≈ ah·bh +
//                     ah·bl + al·bh (3 MFMAs per term, the dropped al·bl and lo's rounding <= 2^-22
//                     relative).  fp16's range is kept by power-of-two per-layer weight scales chosen
//                     at pack time (exact: they fold into the biases and the fp32 output layer), so
//                     small weights' lo parts stay out of fp16 subnormals; an activation beyond fp16's
//                     range makes a non-finite logit, which the kernel counts (ActorOut.ovf,
//                     mdr_actor_status).  MDR_OPT_ACTOR_FP32_FORM = 1 (kernel PREC 6): the three-way
//                     bf16 split x = hi + mid + lo (24 significant bits) and a·b ≈ ah·bh + ah·bm + am·bh
//                     + ah·bl + al·bh + am·bm, 6 MFMAs per term, no range limit.
//   MDR_PREC_BF16   — one bf16 product per term.
// The biases enter as each layer's first accumulator (the MFMA's C operand); ReLU, the output
// layer, softmax and sampling are fp32.
//
// Observation rows.  The rows live in LDS in the chunked slot layout of ActorDims (own features,
// then each message padded to a multiple of 4 floats): in the ring topology one LDS row per message
// source holds that house's message and, for the tile's houses, its own features, so a house's
// message is computed once for the (up to 10) houses that receive it and no row is ever assembled —
// every lane reads its B-fragment chunks with ds_read_b128 straight from the source rows (the
// chunk offsets are per-lane constants).  Table topologies (closed groups, random) gather each
// house's K messages into its own row.
//
// Fragment maps (gfx950, 16x16x32 bf16; lane l, c = l & 15, g = l >> 4, element j = 0..7):
//   A[row c][k = 8g + j], B[k = 8g + j][col c], C/D reg i: col c, row 4g + i.
// Layer 2 takes layer 1's accumulators of row blocks 2q and 2q + 1 directly as its B fragment for
// k-step q: element j is hidden row 32q + 16 (j >> 2) + 4g + (j & 3); the packed W2 fragments use
// that same k order (k_actor_pack), so no lane movement is needed.
#include "mdr_actor.h"
#include "mdr_obs_dev.h"

namespace mdr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// the MFMA operand fragment of a kernel precision: fp16 for the fp16-split form (PREC 4), bf16 otherwise
template <int PREC> struct FragOf { using T = bf16x8; };
template <> struct FragOf<4> { using T = f16x8; };
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// --------------------------------------------------------------------------------------- slots
// The feature behind layer-1 slot s (-1: a padding slot)
__device__ __forceinline__ int actor_feat_of_slot(const ActorDims& d, int s) {
  if (s < d.own4) return s < d.n_own ? s : -1;
  const int t = s - d.own4;
  if (t >= d.n_comm * d.m4) return -1;
  const int k = t / d.m4, m = t - k * d.m4;
  return m < d.msg_w ? d.n_own + k * d.msg_w + m : -1;
}
// Float offset of slot s's value for tile house r, relative to r * rs (-1: padding past the row)
__device__ __forceinline__ int actor_slot_off(const ActorDims& d, int s) {
  if (s >= d.nslot) return -1;
  if (s < d.own4) return d.ring ? d.lo * d.rs + d.m4 + s : s;
  const int t = s - d.own4, k = t / d.m4, m = t - k * d.m4;
  return d.ring ? (k + (k >= d.lo ? 1 : 0)) * d.rs + m : d.own4 + t;
}

// --------------------------------------------------------------------------------------- pack
// One thread per (fragment, lane): 8 weights -> bf16 hi (and lo) in fragment order.
__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (__bf16)v[j];
    lo[j] = (__bf16)(v[j] - (float)hi[j]);
  }
}

__device__ __forceinline__ void split8x3(const float* v, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (__bf16)v[j];
    const float r = v[j] - (float)hi[j];  // exact (Sterbenz / the leading bits cancel)
    mid[j] = (__bf16)r;
    lo[j] = (__bf16)(r - (float)mid[j]);
  }
}

__device__ __forceinline__ bool actor_uniform_feat(const ActorFold& fo, int fe) {
  for (int u = 0; u < fo.nu; ++u)
    if (fo.feat[u] == fe) return true;
  return false;
}

// the packed fragments of one (row block, k-step): nf = 2 (hi, lo) or 3 (hi, mid, lo); d.f16: fp16
// (hi, lo) of the values times the layer's scale (a power of two: exact)
__device__ __forceinline__ void pack_frags(const ActorDims& d, const float* v, unsigned char* base, int f, int lane,
                                           float scale = 1.f) {
  if (d.f16) {
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = v[j] * scale;
      h[j] = (_Float16)x;
      l[j] = (_Float16)(x - (float)h[j]);  // (the difference is exact in fp32)
    }
    f16x8* o = reinterpret_cast<f16x8*>(base);
    o[2 * f * 64 + lane] = h;
    o[(2 * f + 1) * 64 + lane] = l;
    return;
  }
  bf16x8 hi, mid, lo;
  if (d.nf == 3) split8x3(v, hi, mid, lo);
  else split8(v, hi, lo);
  bf16x8* o = reinterpret_cast<bf16x8*>(base);
  o[(d.nf * f) * 64 + lane] = hi;
  if (d.nf == 3) {
    o[(3 * f + 1) * 64 + lane] = mid;
    o[(3 * f + 2) * 64 + lane] = lo;
  } else {
    o[(2 * f + 1) * 64 + lane] = lo;
  }
}

__global__ void k_actor_pack(ActorDims d, ActorFold fo, const float* __restrict__ w1, const float* __restrict__ b1,
                             const float* __restrict__ w2, const float* __restrict__ b2,
                             const float* __restrict__ w3, const float* __restrict__ b3,
                             unsigned char* __restrict__ out) {
  const int nf1 = d.mb * d.ks1, nf2 = d.mb * kActorKS2;
  // fp16 form: the per-layer power-of-two weight scales s1, s2 (every block reduces max |W| itself:
  // ~23k floats).  s = 2^(kActorF16Exp - e) with max |W| < 2^e, so every scaled weight is below
  // 2^kActorF16Exp and weights down to 2^-(kActorF16Exp + 11) of the largest keep their lo part out of
  // fp16 subnormals.  The layer-1 accumulator is then s1 x the reference's, layer 2's s1 s2 x: b1 and
  // b2 are packed scaled alike and W3 by 1 / (s1 s2), so the logits are the reference's.  Layer 2's
  // fp16 operand is relu(layer 1) x s1: s1 is also capped so that the folded bias (b1 + the folded
  // features' contribution, bounded by ActorFold.cfmax) stays below 2^kActorF16Bias, which leaves that
  // operand inside fp16's range while sum |x| over the rest of the obs row stays below
  // (2^15 - 2^kActorF16Bias) / 2^kActorF16Exp; k_actor checks (tile_exact).
  float s1 = 1.f, s2 = 1.f;
  if (d.f16) {
    __shared__ float red[3][256];
    float m1 = 0.f, m2 = 0.f, mb = 0.f;
    for (int i = threadIdx.x; i < d.h1 * d.n_in; i += blockDim.x)
      if (!actor_uniform_feat(fo, i % d.n_in)) m1 = fmaxf(m1, fabsf(w1[i]));  // (folded columns: fp32)
    for (int i = threadIdx.x; i < d.h2 * d.h1; i += blockDim.x) m2 = fmaxf(m2, fabsf(w2[i]));
    for (int i = threadIdx.x; i < d.h1; i += blockDim.x) {  // the folded bias' bound, row i
      float b = fabsf(b1[i]);
      for (int u = 0; u < fo.nu; ++u) b += fabsf(w1[(size_t)i * d.n_in + fo.feat[u]]) * fo.cfmax[u];
      mb = fmaxf(mb, b);
    }
    red[0][threadIdx.x] = m1;
    red[1][threadIdx.x] = m2;
    red[2][threadIdx.x] = mb;
    __syncthreads();
    for (int h = blockDim.x / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h)
        for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = fmaxf(red[k][threadIdx.x], red[k][threadIdx.x + h]);
      __syncthreads();
    }
    int e;
    if (red[0][0] > 0.f && red[0][0] < INFINITY) { frexpf(red[0][0], &e); s1 = ldexpf(1.f, kActorF16Exp - e); }
    if (red[2][0] > 0.f && red[2][0] < INFINITY) {
      frexpf(red[2][0], &e);
      s1 = fminf(s1, ldexpf(1.f, kActorF16Bias - e));
    }
    if (red[1][0] > 0.f && red[1][0] < INFINITY) { frexpf(red[1][0], &e); s2 = ldexpf(1.f, kActorF16Exp - e); }
  }
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = gid & 63, f = gid >> 6;
  const int c = lane & 15, g = lane >> 4;
  float v[8];
  // fragments are stored k-step-major (f = k-step * mb + row block), so the kernel's unrolled
  // (k-step, row block) loops address them with compile-time LDS offsets
  if (f < nf1) {  // W1 [H1][n_in], columns in slot order
    const int ks = f / d.mb, mb = f % d.mb;
    const int row = kActorRB * mb + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int fe = actor_feat_of_slot(d, 32 * ks + 8 * g + j);
      v[j] = (row < d.h1 && fe >= 0 && !(d.f16 && actor_uniform_feat(fo, fe))) ? w1[row * d.n_in + fe] : 0.f;
    }
    pack_frags(d, v, out + d.off_w1, f, lane, s1);
  } else if (f < nf1 + nf2) {  // W2 [H2][H1], fragment (mb, q) in the accumulator k order
    const int f2 = f - nf1;
    const int q = f2 / d.mb, mb = f2 % d.mb;
    const int row = kActorRB * mb + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * q + 16 * (j >> 2) + 4 * g + (j & 3);
      v[j] = (row < d.h2 && k < d.h1) ? w2[row * d.h1 + k] : 0.f;
    }
    pack_frags(d, v, out + d.off_w2, f2, lane, s2);
  } else if (f == nf1 + nf2) {  // fp32 tail: b1, b2 [128], W3^T [128][2] (row-interleaved), b3 [2]
    float* t = reinterpret_cast<float*>(out + d.off_tail);
    const float s12 = s1 * s2, r12 = 1.f / s12;  // (powers of two: exact)
    for (int i = lane; i < kActorRows; i += 64) {
      t[i] = i < d.h1 ? b1[i] * s1 : 0.f;
      t[kActorRows + i] = i < d.h2 ? b2[i] * s12 : 0.f;
      for (int a = 0; a < kActorNA; ++a) t[2 * kActorRows + i * kActorNA + a] = i < d.h2 ? w3[a * d.h2 + i] * r12 : 0.f;
    }
    if (lane < kActorNA) t[(2 + kActorNA) * kActorRows + lane] = b3[lane];
    if (lane == 0) t[kActorTailS1] = s1;
    int* tf = reinterpret_cast<int*>(t + kActorTailFold);  // the folded features (ActorFold)
    if (lane == 0) {
      tf[0] = d.f16 ? fo.nu : 0;
      tf[1] = d.f16 ? fo.nu_own : 0;
    }
    for (int u = lane; u < kActorMaxU; u += 64) {
      tf[2 + u] = fo.feat[u];
      tf[2 + kActorMaxU + u] = fo.cf[u];
    }
  }
}

// --------------------------------------------------------------------------------------- forward
template <typename T = bf16x8>
__device__ __forceinline__ T lds_frag(const unsigned char* base, int frag, int lane) {
  return reinterpret_cast<const T*>(base)[frag * 64 + lane];
}

__device__ __forceinline__ float philox_u01f(uint64_t seed, uint64_t gid, uint64_t tick) {
  const u32x4 c = philox4x32_10(u32x4{(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)tick,
                                      (uint32_t)(tick >> 32) ^ 0xAC7u},
                                (uint32_t)seed ^ 0x3C6EF372u, (uint32_t)(seed >> 32));
  return (float)(c.x >> 8) * (1.0f / 16777216.0f);  // [0, 1), 24 bits
}

// LDS written by some lanes of a wave and read by others: the wave's LDS operations execute in
// issue order, so a wavefront-scope fence (orders the compiler, waits lgkmcnt) is enough.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// max(x, 0) as one v_max_i32 on the bits (fmaxf in IEEE mode adds a quieting v_max per operand):
// every negative float is a negative integer, so it becomes +0; -0 becomes +0; a NaN passes
// through (torch.relu(nan) = nan)
__device__ __forceinline__ float relu(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// acc = C + A·B over the split operands (PREC 1: hi·hi; 3 and 4: + lo terms; 6: + mid terms),
// smallest terms first; a[e] / b[e] = (hi, lo) or (hi, mid, lo)
template <int PREC, typename T>
__device__ __forceinline__ f32x4 mfma_split(const T* a, const T* b, f32x4 acc) {
  if constexpr (PREC == 6) {
    acc = mfma16(a[1], b[1], acc);  // mid·mid
    acc = mfma16(a[2], b[0], acc);  // lo·hi
    acc = mfma16(a[0], b[2], acc);  // hi·lo
    acc = mfma16(a[1], b[0], acc);  // mid·hi
    acc = mfma16(a[0], b[1], acc);  // hi·mid
  } else if constexpr (PREC == 3 || PREC == 4) {
    acc = mfma16(a[1], b[0], acc);  // lo·hi
    acc = mfma16(a[0], b[1], acc);  // hi·lo
  }
  return mfma16(a[0], b[0], acc);
}

// scalar f32 ops the SLP vectorizer cannot pair into v_pk_* (beside MFMAs a v_pk_add_f32 / v_pk_fma_f32
// costs ~22 cycles more than its two scalar halves: MI355X_MICROARCH.md, filler prices)
__device__ __forceinline__ float sub_s(float a, float b) {
  float d;
  asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ float fma_s(float a, float b, float c) {
  float d;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// The per-tile activation split of the bf16x3 form: hi = x with its low 16 bits cleared (a bf16
// value, so its conversion is exact), lo = bf16(x - hi) (the difference is exact).  Truncation
// instead of rounding for hi: two VALU ops per value besides the (co-issued) packing conversions,
// against 2.5 with a rounded hi; |lo| < 2^-7 |x| instead of 2^-8, which leaves the dropped lo·lo
// product below 2^-16 of the term (bf16x3 stays within its 1e-4 probability tolerance).
__device__ __forceinline__ void split8_trunc(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float h = __uint_as_float(__float_as_uint(v[j]) & 0xffff0000u);
    hi[j] = (__bf16)h;
    lo[j] = (__bf16)sub_s(v[j], h);
  }
}

// The fp16-split form's activation split (PREC 4): hi = fp16(x) rounded to nearest, lo = fp16(x - hi)
// (the difference is exact in fp32; |lo| <= 2^-11 |x|, its rounding <= 2^-23 |x|).
__device__ __forceinline__ void split8_f16(const float* v, f16x8& hi, f16x8& lo) {
  // per pair: hi = both values rounded to f16 in one v_cvt_pk_f16_f32 (RNE), each remainder x - hi as
  // one mixed-precision FMA reading its half of the packed hi (v_fma_mix_f32: no conversion back to
  // f32; exact, hi is representable in f32), the remainders packed by a second v_cvt_pk_f16_f32
  uint32_t h[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t hp, lp;
    float d0, d1;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(hp) : "v"(v[2 * q]), "v"(v[2 * q + 1]));
    asm("v_fma_mix_f32 %0, -1.0, %1, %2 op_sel_hi:[0,1,0]" : "=v"(d0) : "v"(hp), "v"(v[2 * q]));
    asm("v_fma_mix_f32 %0, -1.0, %1, %2 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d1) : "v"(hp), "v"(v[2 * q + 1]));
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(lp) : "v"(d0), "v"(d1));
    h[q] = hp;
    l[q] = lp;
  }
  hi = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

template <int PREC, typename T>
__device__ __forceinline__ void split_operand(const float* v, T* s) {
  if constexpr (PREC == 4) split8_f16(v, s[0], s[1]);
  else if constexpr (PREC == 6) split8x3(v, s[0], s[1], s[2]);
  else if constexpr (PREC == 3) split8_trunc(v, s[0], s[1]);  // (r03's rounded-hi split: DESIGN.md §3.4)
  else {
#pragma unroll
    for (int j = 0; j < 8; ++j) s[0][j] = (__bf16)v[j];
  }
}

// The fp16-split form's fallback for a tile whose values leave fp16's range: the logits (without
// b3) of the tile's houses in scalar fp32 from the raw weights [w1 b1 w2 b2 w3 b3] (d.w1raw), the obs
// rows from the tile's LDS rows, one house at a time across the wave — lane j holds hidden neurons j
// and j + 64 of both layers, each a sequential fmaf chain over its inputs (the layer-2 inputs by
// wave broadcast), the logits a wave sum.  The folded features (ActorFold, the packed tail) enter
// through b1f = s1 (b1 + their contribution) / s1 (exact), their row slots / columns skipped.
// Returns house `lane`'s logits on lanes < nb.  Rare (tools: mdr_actor_status 'exact'): ~20 us a tile.
__device__ float2 actor_tile_fp32(const ActorDims& d, const float* w_row, const float* b1f, float s1b,
                                               const float* s_tail, int lane, int nb) {
  const float* W1 = d.w1raw;
  const float* W2 = W1 + (size_t)d.h1 * d.n_in + d.h1;
  const float* B2 = W2 + (size_t)d.h2 * d.h1;
  const float* W3 = B2 + d.h2;
  const int* tf = reinterpret_cast<const int*>(s_tail + kActorTailFold);
  const int nu = tf[0];
  float2 mine = make_float2(0.f, 0.f);
  for (int r = 0; r < nb; ++r) {
    float h1[2], h2[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = lane + 64 * q;
      float a = i < d.h1 ? b1f[i] / s1b : 0.f;
      if (i < d.h1)
        for (int f = 0; f < d.n_in; ++f) {
          bool folded = false;
          for (int k = 0; k < nu; ++k) folded = folded || tf[2 + k] == f;
          if (folded) continue;
          const int s = f < d.n_own ? f : d.own4 + ((f - d.n_own) / d.msg_w) * d.m4 + (f - d.n_own) % d.msg_w;
          a = fmaf(W1[(size_t)i * d.n_in + f], w_row[r * d.rs + actor_slot_off(d, s)], a);
        }
      h1[q] = fmaxf(a, 0.f);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = lane + 64 * q;
      float a = j < d.h2 ? B2[j] : 0.f;
      for (int i = 0; i < d.h1; ++i) {
        const float hv = __shfl(h1[i >> 6], i & 63);
        if (j < d.h2) a = fmaf(W2[(size_t)j * d.h1 + i], hv, a);
      }
      h2[q] = fmaxf(a, 0.f);
    }
    float z0 = 0.f, z1 = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = lane + 64 * q;
      if (j < d.h2) {
        z0 = fmaf(W3[j], h2[q], z0);
        z1 = fmaf(W3[d.h2 + j], h2[q], z1);
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      z0 += __shfl_xor(z0, off);
      z1 += __shfl_xor(z1, off);
    }
    if (lane == r) mine = make_float2(z0, z1);
  }
  return mine;
}

// Persistent: every wave of the block shares the LDS weight image but owns its own 32-house tiles
// (source rows, FSM words in a private LDS slice).  A tile runs as three stages — build (its LDS
// rows from sources prefetched into registers), X (layers 1 and 2 on the MFMA pipe; the next tile's
// sources go in flight first) and Y (output layer, softmax, sampling, stores on the VALU); the
// waves run them free (a ping-pong schedule of the two waves of a SIMD, tried in r03, was slower:
// DESIGN.md §3.4).  MB: row blocks of the hidden layers (compile-time LDS offsets); KS1: layer-1
// k-steps (d.ks1, 2 to 4; no per-step guards in the MFMA loop).  DEF: the reference's default obs
// layout (the 'neighbours' ring, 4-float messages, no optional state or message features), fixed at
// compile time: the optional features' branches and their uniform operands leave the kernel (the
// generic form spills ~127 SGPRs into VGPR lanes, reloaded by v_readlane in the tile loop; DEF 19).
template <int PREC, bool PROF, int MB, int KS1, bool DEF>
__global__ void __launch_bounds__(64 * actor_max_waves(PREC, DEF)) k_actor(KParams p, ObsArgs o, ActorDims d, const double* p_dev,
                                               const unsigned char* __restrict__ wpack, ActorOut out,
                                               uint64_t tick0, const TickArgs* tkp) {
  if (DEF) {  // (the host launches DEF only for this layout: mdr_capi.hip actor_def_layout)
    o.hvac_state = 0; o.solar_state = 0; o.thermal_state = 0; o.msg_thermal = 0; o.msg_hvac = 0;
    o.comm_mode = MDR_COMM_RING; o.msg_w = 4; o.comm_table = nullptr; o.msg_all = nullptr;
    d.ring = 1; d.m4 = 4; d.msg_w = 4; d.n_own = 10; d.own4 = 12; d.rs = 20; d.nf = PREC == 6 ? 3 : 2;
    d.f16 = PREC == 4;
  }
  static_assert(MB >= 1 && MB <= kActorMaxMB, "row blocks");
  static_assert(KS1 >= 1 && KS1 <= kActorMaxSlots / 32, "layer-1 k-steps");
  constexpr int NS = PREC == 6 ? 3 : PREC == 3 || PREC == 4 ? 2 : 1;  // operand splits
  constexpr int NF = PREC == 6 ? 3 : 2;                   // packed fragments per (row block, k-step)
  constexpr int KS2 = (MB + 1) / 2;
  using FragT = typename FragOf<PREC>::T;
  const uint64_t tick = tkp ? tkp->tick : tick0;
  // diagnostics (out.prof): shader cycles per phase, accumulated by lane 0 of every wave:
  // [0] weight fill + block barrier, [1] obs build, [2] prefetch issue + obs_out,
  // [3] layer 1, [4] split + layer 2, [5] output layer + softmax + stores, [6] barrier waits, [7] tiles
  unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long plast = PROF ? clock64() : 0ull;
#define PSTAMP(k)                                \
  do {                                           \
    if (PROF) {                                  \
      const unsigned long long now_ = clock64(); \
      pacc[k] += now_ - plast;                   \
      plast = now_;                              \
    }                                            \
  } while (0)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nthr = blockDim.x, nw = nthr >> 6;
  const int cc = lane & 15, g = lane >> 4;
  const int F = o.n_feat;
  const int K = o.n_comm, M = o.msg_w;
  const bool ring = d.ring != 0;
  const int lo = d.lo, hi = ring ? (K + 1) / 2 : 0;
  const int RS = d.rs;
  const bool thermal = obs_needs_thermal(o);
  const ObsDiv dv = obs_div(p);

  // LDS: [weights image | obs consts | count histogram | per-wave slices]
  const unsigned char* s_w1 = smem;
  const unsigned char* s_w2 = smem + d.off_w2;
  const float* s_tail = reinterpret_cast<const float*>(smem + d.off_tail);
  float* s_cf = reinterpret_cast<float*>(smem + d.lds_cf);
  unsigned* s_hist = reinterpret_cast<unsigned*>(smem + d.lds_hist);
  unsigned char* wbase = smem + d.lds_wave + wv * d.wave_stride;
  float* w_row = reinterpret_cast<float*>(wbase);                  // [nrows][RS]
  uint32_t* w_hw = reinterpret_cast<uint32_t*>(wbase + d.w_hw);    // [32] hvac words
  uint8_t* w_cls = wbase + d.w_cls;                                // [32] capacity classes

  {
    const uint4* src = reinterpret_cast<const uint4*>(wpack);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = d.off_end / 16;
    for (int q = tid; q < n16; q += nthr) {
      if (PREC == 1 && q < d.off_tail / 16 && ((q >> 6) & 1)) continue;  // bf16: no lo fragments (nf = 2)
      dst[q] = src[q];
    }
    // the wave's slice: rows and the zero chunk (padding slots stay zero: the builds write features only)
    for (int q = lane; q < d.w_hw / 4; q += 64) w_row[q] = 0.f;
    if (tid < MDR_MAX_CAP) s_hist[tid] = 0u;
    if (o.sc_dev) { o.s = o.sc_dev[1]; o.solar = o.sc_dev[2]; o.t_od = o.sc_dev[3]; }  // mdr_obs_scalars row
    obs_consts(p, o, p_dev ? *p_dev : o.p, s_cf, tid, nthr);
  }
  __syncthreads();
  // fp16-split form: the layer-1 bias with the house-independent features' contribution (the obs
  // rows hold 0 in their slots), s1 x (b1 + sum_u W1[i][f_u] cf_u) in fp32 from the raw weights (s1
  // keeps it below 2^kActorF16Bias for the features' bounds: k_actor_pack)
  const float* b1 = s_tail;
  const float* b2 = s_tail + kActorRows;
  const float s1b = PREC == 4 ? s_tail[kActorTailS1] : 1.f;  // (the layer-1 accumulator's scale)
  if (PREC == 4) {
    float* s_b1 = reinterpret_cast<float*>(smem + d.lds_b1);
    const int* tf = reinterpret_cast<const int*>(s_tail + kActorTailFold);
    const int nu = tf[0];
    for (int i = tid; i < kActorRows; i += nthr) {
      float u = 0.f;
      if (i < d.h1) {
        const float* wr = d.w1raw + (size_t)i * d.n_in;
        for (int k = 0; k < nu; ++k) u = fmaf(wr[tf[2 + k]], s_cf[tf[2 + kActorMaxU + k]], u);
      }
      s_b1[i] = s_tail[i] + s1b * u;
    }
    __syncthreads();
    b1 = s_b1;
  }
  PSTAMP(0);
  const float* w3 = s_tail + 2 * kActorRows;
  const float* b3 = s_tail + (2 + kActorNA) * kActorRows;

  // this lane's B-fragment chunk addresses (floats into w_row) for column block 0: layer-1 k-step
  // ks reads slots 32 ks + 8 g .. + 7 = two chunks; padding chunks read the wave's zero chunk
  int xoff[KS1][2], xstep[KS1][2];  // column block cb reads xoff + cb * xstep
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int off = actor_slot_off(d, 32 * ks + 8 * g + 4 * e);
      xoff[ks][e] = off < 0 ? d.w_zero / 4 : cc * RS + off;
      xstep[ks][e] = off < 0 ? 0 : 16 * RS;
    }

  const uint32_t n = (uint32_t)p.n;
  const uint32_t ntile = (n + 31u) / 32u;
  const uint32_t stride = gridDim.x * (uint32_t)nw;
  // the launch's tiles as virtual indices v < nv (out.tiles: all, the interior ones, or the first and
  // last — the sharded tick runs the interior while the ring halo is in flight)
  const uint32_t nv = out.tiles == 1 ? ntile - 2u : out.tiles == 2 ? 2u : ntile;
  auto real_tile = [&](uint32_t v) -> uint32_t {
    return out.tiles == 1 ? v + 1u : out.tiles == 2 ? (v == 0u ? 0u : ntile - 1u) : v;
  };
  const int nsrc_max = ring ? lo + 32 + hi : 32;
  HouseRegs src{};
  int src_kind = 0;  // 0 none, 1 house, 2 halo
  // (PREC 4) a row of this lane's current tile holds a seconds-since-off ratio int(sso / L) >= 2^15
  // (a house off for more than 2^15 L seconds: beyond what fp16 carries with room to spare)
  bool xbig = false;
  const uint32_t xthr = dv.L <= 131071u ? 32768u * dv.L : 0xFFFFFFFFu;

  // source s of tile tl: ring = house b0 - lo + s (message source), table = house b0 + s (s < 32)
  auto source_of = [&](uint32_t tl, int s, HouseRegs& rg) -> int {
    const uint32_t b0 = tl * 32u;
    const int nb = (int)min(32u, n - b0);
    if (s >= lo + nb + hi) return 0;
    int64_t j = (int64_t)b0 - lo + s;
    if (o.halo_msg && (j < 0 || j >= (int64_t)n)) return 2;
    if (n >= 64u) {  // j in [-lo, n + 32 + hi): one wrap at most (lo, hi <= 32)
      j = j < 0 ? j + n : (j >= (int64_t)n ? j - n : j);
    } else {
      j %= (int64_t)n;
      if (j < 0) j += n;
    }
    house_load(p, j, thermal, rg);
    return 1;
  };
  auto build = [&](uint32_t b0, int nb, int s, int kind, const HouseRegs& rg) {
    float* row = w_row + s * RS;
    if (kind == 2) {
      const int64_t j = (int64_t)b0 - lo + s;
      const int hh = j < 0 ? (int)(j + lo) : (int)(lo + (j - (int64_t)n));
      const float* src = o.halo_next && hh >= lo ? o.halo_next + (size_t)(hh - lo) * M : o.halo_msg + (size_t)hh * M;
      for (int m = 0; m < M; ++m) row[m] = src[m];
      if (PREC == 4) xbig = xbig || src[1] >= 32768.f;  // (a message's sso ratio, msg_from_regs)
    } else if (kind == 1) {
      if (PREC == 4) xbig = xbig || hv_sso(rg.w) >= xthr;
      const int t = s - lo;
      if (ring) {
        msg_from_regs(p, o, rg, s_cf, row, dv);
        if (t >= 0 && t < nb) row_scalars(p, o, rg, s_cf, row + d.m4, dv, PREC == 4);
      } else {
        row_scalars(p, o, rg, s_cf, row, dv, PREC == 4);
      }
      if (t >= 0 && t < nb) {
        w_hw[t] = rg.w;
        w_cls[t] = (uint8_t)rg.cls;
      }
    }
  };
  // ---- the stages of a tile (build, X, Y: the comment above k_actor)
  f32x2 zz[2];  // the tile's two logits per column block (partial over this lane's rows) between X and Y
  bool tile_exact = false;  // (PREC 4) the tile's values left fp16's range: its outputs come from the fallback pass
  // build: the tile's LDS rows from the prefetched sources (+ the table topologies' gathers)
  auto stage_build = [&](uint32_t tl) {
    const uint32_t b0 = tl * 32u;
    const int nb = (int)min(32u, n - b0);
    wave_sync();  // this wave's previous MFMA-operand reads of the rows are done (compiler ordering)
    xbig = false;
    build(b0, nb, lane, src_kind, src);
    if (nsrc_max > 64 && lane + 64 < lo + nb + hi) {  // rings wider than 32 neighbours
      HouseRegs r2;
      const int k2 = source_of(tl, lane + 64, r2);
      build(b0, nb, lane + 64, k2, r2);
    }
    if (!ring && K > 0) {  // table topologies: lanes r and r + 32 gather half of house r's messages each
      const int r = lane & 31, hh = lane >> 5, kh = (K + 1) / 2;
      if (r < nb) {
        const int64_t i = (int64_t)b0 + r;
        float* row = w_row + r * RS + d.own4;
        for (int k = hh * kh; k < min(K, (hh + 1) * kh); ++k) {
          const int64_t j = o.comm_table[i * K + k];
          if (o.msg_all) {  // sharded: the all-gathered rows, global ids
            for (int m = 0; m < M; ++m) row[k * d.m4 + m] = o.msg_all[j * M + m];
          } else {
            msg_features(p, o, j, s_cf, row + k * d.m4, dv);
          }
          if (PREC == 4) xbig = xbig || row[k * d.m4 + 1] >= 32768.f;  // (the message's sso ratio)
        }
      }
    }
    wave_sync();
    PSTAMP(1);
  };
  // X: the next tile's sources go in flight, then layers 1 and 2 on the MFMA pipe (next >= ntile: none)
  auto stage_x = [&](uint32_t tl, uint32_t next) {
    const uint32_t b0 = tl * 32u;
    const int nb = (int)min(32u, n - b0);
    src_kind = next < ntile ? source_of(next, lane, src) : 0;  // (in flight during the MFMAs)
    if (out.obs) {  // optional obs rows to HBM in the reference's feature order (training buffers)
      float* dst = out.obs + (size_t)b0 * F;
      for (int q = lane; q < nb * F; q += 64) {
        const int rr = q / F, f = q - rr * F;
        const int s = f < d.n_own ? f : d.own4 + ((f - d.n_own) / M) * d.m4 + (f - d.n_own) % M;
        float v = w_row[rr * RS + actor_slot_off(d, s)];
        if (PREC == 4 && f < d.n_own) {  // (the folded own features' slots hold 0: their values)
          const int* tf = reinterpret_cast<const int*>(s_tail + kActorTailFold);
          for (int k = 0; k < tf[1]; ++k)
            if (tf[2 + k] == f) v = s_cf[tf[2 + kActorMaxU + k]];
        }
        dst[q] = v;
      }
      // (these stores' data registers are reused below: the wait here keeps the compiler's wait-count
      // pass from putting one in front of layer 1 on the paths without obs rows)
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), on this path only
    }
    PSTAMP(2);
    // (the wave in its MFMA stage gets VALU issue priority over the SIMD's other wave, which is then
    // building observations or running the output layer)
    __builtin_amdgcn_s_setprio(2);
    // ---- layer 1: acc1 = b1 + W1 · X  (X^T columns = this wave's 32 houses, two column blocks), row
    // block by row block (mb-major: one block's accumulators live at a time); each pair of finished
    // blocks (2q, 2q + 1) becomes layer 2's B fragment of k-step q at once (ReLU + split, VALU work
    // that overlaps the next block's MFMAs).  Weight fragments (packed k-step-major: step (ks, mb) =
    // fragment ks * MB + mb) are read from LDS two steps ahead (a ring of three), so the MFMAs of one
    // wave do not wait out the LDS latency.
    constexpr int PF = 2;  // prefetch distance (steps)
    FragT hs[KS2][2][NS];
    // fp16-split form (PREC 4): layer 2's operand relu(layer 1) must stay inside fp16's range.  Layer 1
    // tracks its maximum (on the bits: non-negative floats order as integers); a tile holding a value
    // >= 2^15, or an input beyond it (xbig), has its logits computed again in scalar fp32 from the raw
    // weights (actor_tile_fp32: rare), which stage Y uses instead (tile_exact).
    {
      uint32_t mbits = 0u;
      FragT xs[KS1][2][NS];
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          float xv[8];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int a = xoff[ks][e] + cb * xstep[ks][e];
            const float4 x = *reinterpret_cast<const float4*>(w_row + a);
            xv[4 * e] = x.x; xv[4 * e + 1] = x.y; xv[4 * e + 2] = x.z; xv[4 * e + 3] = x.w;
          }
          split_operand<PREC>(xv, xs[ks][cb]);
        }
      constexpr int total = KS1 * MB;
      auto frag1 = [&](int s, int e) { return lds_frag<FragT>(s_w1, NF * ((s % KS1) * MB + s / KS1) + e, lane); };
      FragT ring[PF + 1][NS];
#pragma unroll
      for (int q = 0; q < PF; ++q)
#pragma unroll
        for (int e = 0; e < NS; ++e) ring[q][e] = frag1(q, e);
      f32x4 acc1[2][2];  // row blocks 2q, 2q + 1 of the pair in progress
#pragma unroll
      for (int st = 0; st < total; ++st) {
        const int mb = st / KS1, ks = st % KS1;
        if (st + PF < total)
#pragma unroll
          for (int e = 0; e < NS; ++e) ring[(st + PF) % (PF + 1)][e] = frag1(st + PF, e);
        const FragT* as = ring[st % (PF + 1)];
        f32x4* a1 = acc1[mb & 1];
        if (ks == 0) {
          const f32x4 bias = *reinterpret_cast<const f32x4*>(b1 + kActorRB * mb + 4 * g);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) a1[cb] = mfma_split<PREC>(as, xs[ks][cb], bias);
        } else {
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) a1[cb] = mfma_split<PREC>(as, xs[ks][cb], a1[cb]);
        }
        if (ks == KS1 - 1 && ((mb & 1) || mb == MB - 1)) {  // the pair (or the odd last block) is done
          const int q = mb >> 1;
          const bool pair = (mb & 1) != 0;
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[j] = relu(acc1[0][cb][j]);
              v[4 + j] = pair ? relu(acc1[1][cb][j]) : 0.f;
            }
            if (PREC == 4)
#pragma unroll
              for (int j = 0; j < 8; j += 2)
                mbits = max(mbits, max(__float_as_uint(v[j]), __float_as_uint(v[j + 1])));
            split_operand<PREC>(v, hs[q][cb]);
          }
        }
      }
      if constexpr (PREC == 4) {
        tile_exact = __ballot(xbig || mbits >= 0x47000000u) != 0ull;  // (>= 2^15 = 32768.0f)
        // (such a tile's outputs are written after the wave's other tiles: the fallback pass below)
      }
    }
    PSTAMP(3);

    // ---- layer 2 (acc2 = b2 + W2 · relu(H1)) fused with the output layer, row block by row block:
    // as soon as a block's four k-steps are done its ReLU'd rows enter the two logits (scalar fp32
    // FMAs in block / row order) while the next block's MFMAs run (not for a tile_exact tile)
    if (!(PREC == 4 && tile_exact)) {
      constexpr int TOT = KS2 * MB;
      auto frag2 = [&](int s, int e) { return lds_frag<FragT>(s_w2, NF * ((s % KS2) * MB + s / KS2) + e, lane); };
      FragT ring[PF + 1][NS];
#pragma unroll
      for (int q = 0; q < PF; ++q)
#pragma unroll
        for (int e = 0; e < NS; ++e) ring[q][e] = frag2(q, e);
      f32x4 acc2[2];
      zz[0] = f32x2{0.f, 0.f};
      zz[1] = f32x2{0.f, 0.f};
#pragma unroll
      for (int st = 0; st < TOT; ++st) {
        const int mb = st / KS2, q = st % KS2;
        if (st + PF < TOT)
#pragma unroll
          for (int e = 0; e < NS; ++e) ring[(st + PF) % (PF + 1)][e] = frag2(st + PF, e);
        const FragT* as = ring[st % (PF + 1)];
        if (q == 0) {
          const f32x4 bias = *reinterpret_cast<const f32x4*>(b2 + kActorRB * mb + 4 * g);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) acc2[cb] = mfma_split<PREC>(as, hs[q][cb], bias);
        } else {
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) acc2[cb] = mfma_split<PREC>(as, hs[q][cb], acc2[cb]);
        }
        if (q == KS2 - 1) {
          const f32x2* wr = reinterpret_cast<const f32x2*>(w3 + (kActorRB * mb + 4 * g) * kActorNA);  // rows 4g .. 4g + 3
          f32x2 w[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = wr[i];
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float x = relu(acc2[cb][i]);
              zz[cb].x = fma_s(w[i].x, x, zz[cb].x);
              zz[cb].y = fma_s(w[i].y, x, zz[cb].y);
            }
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    PSTAMP(4);
  };
  // Y: output layer (fp32 VALU) + softmax + sampling + stores (+ the ON counts of the new actions)
  float u_next = 0.f;  // the sampling uniforms of this wave's next tile (stage_y, odd tiles)
  // skip: the tile's outputs come later (a tile_exact tile in the main loop; its uniforms for the next
  // tile are still drawn)
  // exact: the logits are zx (the fallback pass), lanes < 32 (house = lane)
  auto stage_y = [&](uint32_t tl, uint32_t next, bool fresh, bool skip, bool exact, float2 zx) {
    const uint32_t b0 = tl * 32u;
    const int nb = (int)min(32u, n - b0);
    float z[2][kActorNA];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) { z[cb][0] = zz[cb].x; z[cb][1] = zz[cb].y; }

#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int a = 0; a < kActorNA; ++a) {
        z[cb][a] += __shfl_xor(z[cb][a], 16);
        z[cb][a] += __shfl_xor(z[cb][a], 32);
      }
    // lane l < 32 takes house l (column block l >> 4, column l & 15)
    const int r = lane & 31;
    const bool upper = (lane & 16) != 0;
    const float z0 = (PREC == 4 && exact ? zx.x : upper ? z[1][0] : z[0][0]) + b3[0];
    const float z1 = (PREC == 4 && exact ? zx.y : upper ? z[1][1] : z[0][1]) + b3[1];
    // softmax over the 2 actions (fp32, max-subtracted like torch; one reciprocal of the sum, as
    // ATen's vectorised softmax) + Categorical sample
    const float zmax = fmaxf(z0, z1);
    const float e0 = __expf(z0 - zmax), e1 = __expf(z1 - zmax);
    const float rse = 1.f / (e0 + e1);
    const float p0 = e0 * rse, p1 = e1 * rse;
    const bool valid = r < nb;
    const uint32_t i = b0 + (uint32_t)r;
    // Categorical(probs).sample(): action 0 iff u < p0.  The uniform of house i is
    // philox(seed, goff + i, tick); every other tile, lanes 32..63 draw the next tile's (the same
    // counters: one Philox pass per two tiles), kept in u_next
    float u;
    if (fresh) {
      const uint32_t ih = (lane < 32 ? b0 : next * 32u) + (uint32_t)r;
      u = philox_u01f(p.seed, (uint64_t)p.goff + ih, tick);
      u_next = __shfl(u, r + 32);
    } else {
      u = u_next;
    }
    const int act = u < p0 ? 0 : 1;
    const float pa = act ? p1 : p0;
    const bool writer = valid && lane < 32 && !skip;
    if (PREC == 4 && out.ovf) {  // a non-finite logit (mdr_actor_status)
      const bool bad = writer && !(__builtin_isfinite(z0) && __builtin_isfinite(z1));
      if (__ballot(bad) && lane == 0) atomicAdd(out.ovf, 1u);
    }
    if (writer) {
      if (out.probs) *reinterpret_cast<float2*>(out.probs + 2 * (size_t)i) = make_float2(p0, p1);
      if (out.action) out.action[i] = (uint8_t)act;
      if (out.prob) out.prob[i] = pa;
    }
    if (out.count_next) {
      // the ON houses the new actions produce (hvac.py:43-64 on action != 0), per capacity class
      const bool on1 = writer && hv_on(hvac_fsm(w_hw[r], act != 0, p.dt, p.L));
      const int cls = valid ? w_cls[r] : 0;
      for (int k = 0; k < p.n_cap; ++k) {
        const unsigned long long m = __ballot(on1 && cls == k);
        if (lane == 0 && m) atomicAdd(&s_hist[k], (unsigned)__popcll(m));
      }
    }
    PSTAMP(5);
  };

  // ---- the wave's tiles: build(t0) | X(t0) | Y(t0) + build(t1) | X(t1) | ... | Y(t_last)
  const uint32_t v0 = blockIdx.x * (uint32_t)nw + (uint32_t)wv;
  const int n_my = v0 < nv ? (int)((nv - 1u - v0) / stride + 1u) : 0;
  if (n_my > 0) {
    src_kind = source_of(real_tile(v0), lane, src);
    stage_build(real_tile(v0));
  }
  // the first build's loads have all landed (on every path): the compiler's wait-count pass otherwise
  // carries them, pending on the lanes that skipped the build, into the tile loop and puts an
  // s_waitcnt vmcnt(0) in front of layer 1 on every tile, which also waits for the next tile's
  // prefetch loads just issued (measured: no change of the kernel time, 117.9 vs 118.7-119.4 us —
  // the other waves of the SIMD cover that wait; kept because the wait has no purpose)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  uint64_t exact_tiles = 0ull;  // (PREC 4) the wave's tiles j left to the fallback pass (bit j)
  for (int j = 0; j < n_my; ++j) {
    const uint32_t vj = v0 + (uint32_t)j * stride;
    const uint32_t tj = real_tile(vj);
    const uint32_t next = vj + stride < nv ? real_tile(vj + stride) : ntile;  // (ntile: none)
    if (PROF && lane == 0) pacc[7] += 1;
    stage_x(tj, next);
    const bool defer = PREC == 4 && tile_exact && j < 64;
    if (PREC == 4 && tile_exact && !defer && lane == 0 && out.ovf) atomicAdd(out.ovf, 1u);  // (> 64 tiles a wave)
    if (defer) exact_tiles |= 1ull << j;
    stage_y(tj, next, (j & 1) == 0, defer, false, make_float2(0.f, 0.f));
    if (j + 1 < n_my) stage_build(next);
  }
  // (PREC 4) the fallback pass: each deferred tile's rows built again, its logits in scalar fp32 from
  // the raw weights (actor_tile_fp32), then stage Y with fresh uniforms.  After the tile loop, so
  // the loop's registers are free for it.
  if (PREC == 4)
    while (exact_tiles) {  // (wave-uniform)
      const int j = __ffsll((long long)exact_tiles) - 1;
      exact_tiles &= exact_tiles - 1ull;
      const uint32_t tj = real_tile(v0 + (uint32_t)j * stride);
      src_kind = source_of(tj, lane, src);
      stage_build(tj);
      const float2 zx = actor_tile_fp32(d, w_row, b1, s1b, s_tail, lane, (int)min(32u, n - tj * 32u));
      stage_y(tj, ntile, true, false, true, zx);
      if (lane == 0 && out.ovf) atomicAdd(out.ovf + 1, 1u);  // (mdr_actor_status 'exact')
    }
  if (PROF && lane == 0) {
    for (int k = 0; k < 8; ++k) out.prof[(blockIdx.x * nw + wv) * 8 + k] = pacc[k];
  }
  if (out.count_next) {
    __syncthreads();
    if (tid < p.n_cap && s_hist[tid])
      atomicAdd(&out.count_next[(blockIdx.x % kCountShards) * p.n_cap + tid], (unsigned long long)s_hist[tid]);
  }
#undef PSTAMP
}

// --------------------------------------------------------------------------------------- chain
// The general actor (any number of hidden layers, any widths, any obs row; and the fp32 mode where
// the fused kernel's three weight planes do not fit the LDS): the reference Actor.forward
// (network.py:29-33) as a chain of launches over fp32 rows in HBM — the obs rows (k_obs), one
// k_dense per hidden layer, then k_actor_head (output layer, softmax, sampling, ON counts).  The
// same split-bf16 MFMA products per precision as k_actor, the same sampling stream.

// Y[i][o] = act(b[o] + sum_k W[o][k] X[i][k]) for houses i < n and neurons o < out (row-major fp32,
// leading dimensions ldx / ldy).  A block of 4 waves covers 64 houses x 64 neurons; wave w owns
// neurons 16 w .. 16 w + 15 (the rows of one 16x16x32 MFMA) against four column blocks of 16
// houses; k-steps of 32 with zero-filled edges.  The bias is the first MFMA's C operand.
template <int PREC>
__global__ void __launch_bounds__(256) k_dense(const float* __restrict__ X, int ldx, int K, int64_t n,
                                               const float* __restrict__ W, const float* __restrict__ b, int out,
                                               float* __restrict__ Y, int ldy, int relu_on) {
  constexpr int NS = PREC == 6 ? 3 : PREC == 3 ? 2 : 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int64_t h0 = (int64_t)blockIdx.x * 64;
  const int o0 = ((int)blockIdx.y * 4 + wv) * kActorRB;
  if (o0 >= out) return;  // (wave-uniform)
  const int orow = o0 + c;
  f32x4 bias;
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = o0 + 4 * g + i < out ? b[o0 + 4 * g + i] : 0.f;
  f32x4 acc[4] = {bias, bias, bias, bias};
  for (int k0 = 0; k0 < K; k0 += 32) {
    float av[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + 8 * g + j;
      av[j] = orow < out && k < K ? W[(int64_t)orow * K + k] : 0.f;
    }
    bf16x8 as[NS];
    split_operand<PREC>(av, as);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int64_t hi = h0 + 16 * cb + c;
      float xv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + 8 * g + j;
        xv[j] = hi < n && k < K ? X[hi * ldx + k] : 0.f;
      }
      bf16x8 xs[NS];
      split_operand<PREC>(xv, xs);
      acc[cb] = mfma_split<PREC>(as, xs, acc[cb]);
    }
  }
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int64_t hi = h0 + 16 * cb + c;
    if (hi >= n) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = o0 + 4 * g + i;
      if (o < out) Y[hi * ldy + o] = relu_on ? relu(acc[cb][i]) : acc[cb][i];
    }
  }
}

// The output layer (fp32 FMAs over the last hidden layer, W3 [2][K] row-major, b3 [2]), softmax and
// Categorical sampling of k_actor's stage Y — the same uniform philox(seed, goff + i, tick) per
// house — the stores, and the ON counts of the new actions; one thread per house.
__global__ void __launch_bounds__(256) k_actor_head(KParams p, const float* __restrict__ X, int ldx, int K,
                                                    const float* __restrict__ W3, const float* __restrict__ b3,
                                                    uint64_t tick0, const TickArgs* tkp, ActorOut out) {
  __shared__ unsigned s_hist[MDR_MAX_CAP];
  if (threadIdx.x < MDR_MAX_CAP) s_hist[threadIdx.x] = 0u;
  __syncthreads();
  const uint64_t tick = tkp ? tkp->tick : tick0;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < p.n;
  float z0 = 0.f, z1 = 0.f;
  if (valid) {
    const float* x = X + i * ldx;
    for (int k = 0; k < K; ++k) {
      const float v = x[k];
      z0 = fmaf(W3[k], v, z0);
      z1 = fmaf(W3[K + k], v, z1);
    }
  }
  z0 += b3[0];
  z1 += b3[1];
  const float zmax = fmaxf(z0, z1);
  const float e0 = __expf(z0 - zmax), e1 = __expf(z1 - zmax);
  const float rse = 1.f / (e0 + e1);
  const float p0 = e0 * rse, p1 = e1 * rse;
  const float u = philox_u01f(p.seed, (uint64_t)p.goff + (uint64_t)(valid ? i : 0), tick);
  const int act = u < p0 ? 0 : 1;
  if (valid) {
    if (out.probs) *reinterpret_cast<float2*>(out.probs + 2 * (size_t)i) = make_float2(p0, p1);
    if (out.action) out.action[i] = (uint8_t)act;
    if (out.prob) out.prob[i] = act ? p1 : p0;
  }
  if (out.count_next) {
    const bool on1 = valid && hv_on(hvac_fsm(p.hvac[i], act != 0, p.dt, p.L));
    const int cls = valid ? p.cap_idx[i] : 0;
    for (int k = 0; k < p.n_cap; ++k) {
      const unsigned long long m = __ballot(on1 && cls == k);
      if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_hist[k], (unsigned)__popcll(m));
    }
    __syncthreads();
    if ((int)threadIdx.x < p.n_cap && s_hist[threadIdx.x])
      atomicAdd(&out.count_next[(blockIdx.x % kCountShards) * p.n_cap + threadIdx.x],
                (unsigned long long)s_hist[threadIdx.x]);
  }
}

template __global__ void k_dense<1>(const float*, int, int, int64_t, const float*, const float*, int, float*, int, int);
template __global__ void k_dense<3>(const float*, int, int, int64_t, const float*, const float*, int, float*, int, int);
template __global__ void k_dense<6>(const float*, int, int, int64_t, const float*, const float*, int, float*, int, int);

#define MDR_INST_ACTOR_D(P, F, MB, KS, DF)                                                            \
  template __global__ void k_actor<P, F, MB, KS, DF>(KParams, ObsArgs, ActorDims, const double*,          \
                                                     const unsigned char*, ActorOut, uint64_t, const TickArgs*);
#define MDR_INST_ACTOR(P, F, MB, KS) MDR_INST_ACTOR_D(P, F, MB, KS, false)
#define MDR_INST_ACTOR_SHAPE(MB, KS) \
  MDR_INST_ACTOR(1, false, MB, KS) \
  MDR_INST_ACTOR(3, false, MB, KS) \
  MDR_INST_ACTOR(4, false, MB, KS) \
  MDR_INST_ACTOR(6, false, MB, KS) \
  MDR_INST_ACTOR(1, true, MB, KS)  \
  MDR_INST_ACTOR(3, true, MB, KS)  \
  MDR_INST_ACTOR(4, true, MB, KS)  \
  MDR_INST_ACTOR(6, true, MB, KS)
MDR_INST_ACTOR_SHAPE(7, 2)
MDR_INST_ACTOR_SHAPE(7, 3)
MDR_INST_ACTOR_SHAPE(7, 4)
MDR_INST_ACTOR_SHAPE(8, 2)
MDR_INST_ACTOR_SHAPE(8, 3)
MDR_INST_ACTOR_SHAPE(8, 4)
#define MDR_INST_ACTOR_DEF(MB)                                                                      \
  MDR_INST_ACTOR_D(1, false, MB, 2, true) MDR_INST_ACTOR_D(3, false, MB, 2, true)                   \
  MDR_INST_ACTOR_D(4, false, MB, 2, true) MDR_INST_ACTOR_D(6, false, MB, 2, true)                   \
  MDR_INST_ACTOR_D(1, true, MB, 2, true) MDR_INST_ACTOR_D(3, true, MB, 2, true)                     \
  MDR_INST_ACTOR_D(4, true, MB, 2, true) MDR_INST_ACTOR_D(6, true, MB, 2, true)
MDR_INST_ACTOR_DEF(7)
MDR_INST_ACTOR_DEF(8)

}  // namespace mdr
