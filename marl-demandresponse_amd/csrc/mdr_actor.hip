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
//   MDR_PREC_FP32   — three-way split x = hi + mid + lo (24 significant bits: the whole fp32
//                     significand) and a·b ≈ ah·bh + ah·bm + am·bh + ah·bl + al·bh + am·bm (the dropped
//                     terms are <= 2^-24 relative): fp32-faithful, 6 MFMAs per term.
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

__device__ __forceinline__ void split8x3(const float* v, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (__bf16)v[j];
    const float r = v[j] - (float)hi[j];  // exact (Sterbenz / the leading bits cancel)
    mid[j] = (__bf16)r;
    lo[j] = (__bf16)(r - (float)mid[j]);
  }
}

// the packed fragments of one (row block, k-step): nf = 2 (hi, lo) or 3 (hi, mid, lo)
__device__ __forceinline__ void pack_frags(const ActorDims& d, const float* v, unsigned char* base, int f, int lane) {
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

__global__ void k_actor_pack(ActorDims d, const float* __restrict__ w1, const float* __restrict__ b1,
                             const float* __restrict__ w2, const float* __restrict__ b2,
                             const float* __restrict__ w3, const float* __restrict__ b3,
                             unsigned char* __restrict__ out) {
  const int nf1 = kActorMB * d.ks1, nf2 = kActorMB * d.ks2;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = g & 63, f = g >> 6;
  const int r = lane & 31, h = lane >> 5;
  float v[8];
  // fragments are stored k-step-major (f = k-step * kActorMB + mb), so the kernel's unrolled
  // (k-step, mb) loops address them with compile-time LDS offsets whatever ks1 / ks2 are
  if (f < nf1) {  // W1 [H1][n_in], fragment (mb, ks)
    const int ks = f / kActorMB, mb = f % kActorMB;
    const int row = 32 * mb + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * ks + 8 * h + j;
      v[j] = (row < d.h1 && k < d.n_in) ? w1[row * d.n_in + k] : 0.f;
    }
    pack_frags(d, v, out + d.off_w1, f, lane);
  } else if (f < nf1 + nf2) {  // W2 [H2][H1], fragment (mb, q) in the accumulator k order
    const int f2 = f - nf1;
    const int q = f2 / kActorMB, mb = f2 % kActorMB;
    const int row = 32 * mb + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * q + 8 * (j >> 2) + 4 * h + (j & 3);
      v[j] = (row < d.h2 && k < d.h1) ? w2[row * d.h1 + k] : 0.f;
    }
    pack_frags(d, v, out + d.off_w2, f2, lane);
  } else if (f == nf1 + nf2) {  // fp32 tail: b1, b2 [128], W3^T [128][2] (row-interleaved), b3 [2]
    float* t = reinterpret_cast<float*>(out + d.off_tail);
    for (int i = lane; i < kActorRows; i += 64) {
      t[i] = i < d.h1 ? b1[i] : 0.f;
      t[kActorRows + i] = i < d.h2 ? b2[i] : 0.f;
      for (int a = 0; a < kActorNA; ++a) t[2 * kActorRows + i * kActorNA + a] = i < d.h2 ? w3[a * d.h2 + i] : 0.f;
    }
    if (lane < kActorNA) t[(2 + kActorNA) * kActorRows + lane] = b3[lane];
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

// LDS written by some lanes of a wave and read by others: the wave's LDS operations execute in
// issue order, so a wavefront-scope fence (orders the compiler, waits lgkmcnt) is enough.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Persistent, wave-independent: every wave of the block shares the LDS weight image but owns its
// own 32-house tiles (rows, ring messages, FSM words in a private LDS slice), so waves never wait
// for each other inside the loop and one wave's obs build / memory phase overlaps another's MFMAs
// on the same SIMD.  Each lane prefetches one obs source of the wave's NEXT tile into registers
// before the current tile's MFMAs.
template <int PREC, bool PROF>
__global__ void __launch_bounds__(512) k_actor(KParams p, ObsArgs o, ActorDims d, const double* p_dev,
                                               const unsigned char* __restrict__ wpack, ActorOut out,
                                               uint64_t tick0, const TickArgs* tkp) {
  const uint64_t tick = tkp ? tkp->tick : tick0;
  // diagnostics (out.prof): shader cycles per phase, accumulated by lane 0 of every wave:
  // [0] weight fill + block barrier, [1] obs build + message copy, [2] prefetch issue + obs_out,
  // [3] layer 1, [4] split + layer 2, [5] output layer + softmax + stores, [6] -, [7] tiles
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
  const int r = lane & 31, h = lane >> 5;
  const int F = o.n_feat, FS = d.fs;
  constexpr int NF = PREC == 6 ? 3 : 2;  // packed fragments per (row block, k-step)
  const int K = o.n_comm, M = o.msg_w;
  const bool ring = o.comm_mode == MDR_COMM_RING && K > 0;
  const int lo = ring ? K / 2 : 0, hi = ring ? (K + 1) / 2 : 0;
  const bool thermal = obs_needs_thermal(o);

  // LDS: [weights image | obs consts | count histogram | per-wave slices]
  const unsigned char* s_w1 = smem;
  const unsigned char* s_w2 = smem + d.off_w2;
  const float* s_tail = reinterpret_cast<const float*>(smem + d.off_tail);
  float* s_cf = reinterpret_cast<float*>(smem + d.lds_cf);
  unsigned* s_hist = reinterpret_cast<unsigned*>(smem + d.lds_hist);
  unsigned char* wbase = smem + d.lds_wave + wv * d.wave_stride;
  float* w_obs = reinterpret_cast<float*>(wbase);                  // [32][FS] + 16 ks1 overrun
  float* w_msg = reinterpret_cast<float*>(wbase + d.w_msg);        // [lo + 32 + hi][M]
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
    for (int q = lane; q < 32 * FS + 16 * d.ks1; q += 64) w_obs[q] = 0.f;
    if (tid < MDR_MAX_CAP) s_hist[tid] = 0u;
    if (o.sc_dev) { o.s = o.sc_dev[1]; o.solar = o.sc_dev[2]; o.t_od = o.sc_dev[3]; }  // mdr_obs_scalars row
    obs_consts(p, o, p_dev ? *p_dev : o.p, s_cf, tid, nthr);
  }
  __syncthreads();
  PSTAMP(0);
  const float* b1 = s_tail;
  const float* b2 = s_tail + kActorRows;
  const float* w3 = s_tail + 2 * kActorRows;
  const float* b3 = s_tail + (2 + kActorNA) * kActorRows;

  const uint32_t n = (uint32_t)p.n;
  const uint32_t ntile = (n + 31u) / 32u;
  const uint32_t stride = gridDim.x * (uint32_t)nw;
  const int nsrc_max = lo + 32 + hi;
  HouseRegs src{};
  int src_kind = 0;  // 0 none, 1 house, 2 halo
  auto source_of = [&](uint32_t tl, int s, HouseRegs& rg) -> int {
    const uint32_t b0 = tl * 32u;
    const int nb = (int)min(32u, n - b0);
    if (s >= lo + nb + hi) return 0;
    int64_t j = (int64_t)b0 - lo + s;
    if (o.halo_msg && (j < 0 || j >= (int64_t)n)) return 2;
    j %= (int64_t)n;
    if (j < 0) j += n;
    house_load(p, j, thermal, rg);
    return 1;
  };
  auto build = [&](uint32_t b0, int nb, int s, int kind, const HouseRegs& rg) {
    if (kind == 2) {
      const int64_t j = (int64_t)b0 - lo + s;
      const int hh = j < 0 ? (int)(j + lo) : (int)(lo + (j - (int64_t)n));
      for (int m = 0; m < M; ++m) w_msg[s * M + m] = o.halo_msg[hh * M + m];
    } else if (kind == 1) {
      if (ring) msg_from_regs(p, o, rg, s_cf, w_msg + s * M);
      const int t = s - lo;
      if (t >= 0 && t < nb) {
        float* row = w_obs + t * FS;
        const int f = row_scalars(p, o, rg, s_cf, row);
        if (!ring) row_messages(p, o, (int64_t)b0 + t, t, s_cf, w_msg, row, f);  // TABLE gathers / none
        for (int q = F; q < FS; ++q) row[q] = 0.f;
        w_hw[t] = rg.w;
        w_cls[t] = (uint8_t)rg.cls;
      }
    }
  };
  uint32_t tile = blockIdx.x * (uint32_t)nw + (uint32_t)wv;
  if (tile < ntile) src_kind = source_of(tile, lane, src);

  for (; tile < ntile; tile += stride) {
    const uint32_t b0 = tile * 32u;
    const int nb = (int)min(32u, n - b0);
    if (PROF && lane == 0) pacc[7] += 1;
    wave_sync();  // this wave's previous MFMA reads of w_obs are done (compiler ordering)
    build(b0, nb, lane, src_kind, src);
    if (nsrc_max > 64 && lane + 64 < lo + nb + hi) {  // rings wider than 32 neighbours
      HouseRegs r2;
      const int k2 = source_of(tile, lane + 64, r2);
      build(b0, nb, lane + 64, k2, r2);
    }
    wave_sync();
    if (ring) {  // messages into the rows: lanes r and r + 32 each copy half of row r's K messages
      const int base = F - K * M;
      const int kh = (K + 1) / 2;
      if (r < nb) {
        for (int k = h * kh; k < min(K, (h + 1) * kh); ++k) {
          const int sidx = k < lo ? (r + k) : (r + k + 1);
          float* dst = w_obs + r * FS + base + k * M;
          const float* sp = w_msg + sidx * M;
          for (int m = 0; m < M; ++m) dst[m] = sp[m];
        }
      }
      wave_sync();
    }
    PSTAMP(1);
    if (tile + stride < ntile) src_kind = source_of(tile + stride, lane, src);  // in flight during the MFMAs
    else src_kind = 0;
    if (out.obs) {  // optional obs rows to HBM (training buffers)
      float* dst = out.obs + (size_t)b0 * F;
      for (int q = lane; q < nb * F; q += 64) {
        const int rr = q / F;
        dst[q] = w_obs[rr * FS + (q - rr * F)];
      }
    }
    PSTAMP(2);

    // ---- layer 1: acc1[mb] = b1 + W1 · X  (X^T columns = this wave's 32 houses)
    // (the wave in its MFMA phases gets issue priority over the SIMD's other wave, which is then
    // building observations or running the output layer on the VALU: C5 actor 151 -> 141 us at 1M)
    __builtin_amdgcn_s_setprio(3);
    const float* xrow = w_obs + r * FS + 8 * h;
    f32x16 acc1[kActorMB];
#pragma unroll
    for (int mb = 0; mb < kActorMB; ++mb)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc1[mb][g] = b1[32 * mb + (g & 3) + 8 * (g >> 2) + 4 * h];
    // k-steps unrolled with uniform guards (a loop here makes the compiler drain the prefetch
    // loads, vmcnt(0), at its header)
#pragma unroll
    for (int ks = 0; ks < kActorMaxIn / 16; ++ks) {
      if (ks >= d.ks1) break;
      const float4 x0 = *reinterpret_cast<const float4*>(xrow + 16 * ks);
      const float4 x1 = *reinterpret_cast<const float4*>(xrow + 16 * ks + 4);
      const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 xh, xl, xm;
      if (PREC == 6) split8x3(xv, xh, xm, xl);
      else split8(xv, xh, xl);
      bf16x8 ah[kActorMB], al[kActorMB], am[kActorMB];
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb) {
        const int f = ks * kActorMB + mb;
        ah[mb] = lds_frag(s_w1, NF * f, lane);
        if (PREC == 3) al[mb] = lds_frag(s_w1, NF * f + 1, lane);
        if (PREC == 6) { am[mb] = lds_frag(s_w1, NF * f + 1, lane); al[mb] = lds_frag(s_w1, NF * f + 2, lane); }
      }
      if (PREC == 6) {  // smallest terms first
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mb], xm, acc1[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mb], xh, acc1[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], xl, acc1[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mb], xh, acc1[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc1[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], xm, acc1[mb], 0, 0, 0);
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
    PSTAMP(3);

    // ---- ReLU + split: layer 1's accumulators become layer 2's B fragments in place
    bf16x8 hh[2 * kActorMB], hl[2 * kActorMB], hm[PREC == 6 ? 2 * kActorMB : 1];
#pragma unroll
    for (int q = 0; q < 2 * kActorMB; ++q) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(acc1[q >> 1][8 * (q & 1) + j], 0.f);
      if constexpr (PREC == 6) split8x3(v, hh[q], hm[q], hl[q]);
      else split8(v, hh[q], hl[q]);
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
      bf16x8 ah[kActorMB], al[kActorMB], am[kActorMB];
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb) {
        const int f = q * kActorMB + mb;
        ah[mb] = lds_frag(s_w2, NF * f, lane);
        if (PREC == 3) al[mb] = lds_frag(s_w2, NF * f + 1, lane);
        if (PREC == 6) { am[mb] = lds_frag(s_w2, NF * f + 1, lane); al[mb] = lds_frag(s_w2, NF * f + 2, lane); }
      }
      if constexpr (PREC == 6) {  // smallest terms first
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mb], hm[q], acc2[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mb], hh[q], acc2[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], hl[q], acc2[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mb], hh[q], acc2[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < kActorMB; ++mb) acc2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mb], hm[q], acc2[mb], 0, 0, 0);
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
    __builtin_amdgcn_s_setprio(0);
    PSTAMP(4);

    // ---- output layer (fp32 VALU): this lane's 64 hidden rows, then the partner half's
    float z0 = 0.f, z1 = 0.f;
    {
#pragma clang fp contract(fast)
#pragma unroll
      for (int mb = 0; mb < kActorMB; ++mb)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int row = 32 * mb + (g & 3) + 8 * (g >> 2) + 4 * h;
          const float x = fmaxf(acc2[mb][g], 0.f);
          const float2 w = *reinterpret_cast<const float2*>(w3 + row * kActorNA);
          z0 += w.x * x;
          z1 += w.y * x;
        }
    }
    z0 = z0 + __shfl_xor(z0, 32) + b3[0];
    z1 = z1 + __shfl_xor(z1, 32) + b3[1];

    // ---- softmax over the 2 actions (fp32, max-subtracted like torch) + Categorical sample
    const float zmax = fmaxf(z0, z1);
    const float e0 = expf(z0 - zmax), e1 = expf(z1 - zmax);
    const float se = e0 + e1;
    const float p0 = e0 / se, p1 = e1 / se;
    const bool valid = r < nb;
    const uint32_t i = b0 + (uint32_t)r;
    // Categorical(probs).sample(): action 0 iff u < p0
    const float u = philox_u01f(p.seed, (uint64_t)p.goff + i, tick);
    const int act = u < p0 ? 0 : 1;
    const float pa = act ? p1 : p0;
    if (valid && h == 0) {
      if (out.probs) *reinterpret_cast<float2*>(out.probs + 2 * (size_t)i) = make_float2(p0, p1);
      if (out.action) out.action[i] = (uint8_t)act;
      if (out.prob) out.prob[i] = pa;
    }
    if (out.count_next) {
      // the ON houses the new actions produce (hvac.py:43-64 on action != 0), per capacity class
      const bool on1 = valid && h == 0 && hv_on(hvac_fsm(w_hw[r], act != 0, p.dt, p.L));
      const int cls = valid ? w_cls[r] : 0;
      for (int k = 0; k < p.n_cap; ++k) {
        const unsigned long long m = __ballot(on1 && cls == k);
        if (lane == 0 && m) atomicAdd(&s_hist[k], (unsigned)__popcll(m));
      }
    }
    PSTAMP(5);
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

#define MDR_INST_ACTOR(P, F)                                                                   \
  template __global__ void k_actor<P, F>(KParams, ObsArgs, ActorDims, const double*, const unsigned char*, \
                                         ActorOut, uint64_t, const TickArgs*);
MDR_INST_ACTOR(1, false)
MDR_INST_ACTOR(3, false)
MDR_INST_ACTOR(6, false)
MDR_INST_ACTOR(1, true)
MDR_INST_ACTOR(3, true)
MDR_INST_ACTOR(6, true)

}  // namespace mdr
