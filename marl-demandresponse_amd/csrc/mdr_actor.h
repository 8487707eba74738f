// mdr_actor.h — parameter blocks of the fused obs + MA-PPO actor kernels (mdr_actor.hip).
#pragma once
#include "mdr_kernels.h"

namespace mdr {

constexpr int kActorRB = 16;      // rows (neurons) per MFMA row block (v_mfma_f32_16x16x32_bf16)
constexpr int kActorMaxMB = 8;    // row blocks per hidden layer (hidden width <= 128)
constexpr int kActorRows = kActorRB * kActorMaxMB;
constexpr int kActorNA = 2;       // actions: on / off (MAPPO num_action = 2, mappo.py:38)
constexpr int kActorMaxIn = 128;  // obs features
constexpr int kActorMaxSlots = 128;  // feature slots of the chunked row layout (4 k-steps of 32)
constexpr int kActorKS2 = kActorMaxMB / 2;  // layer-2 k-steps of 32 (hidden rows 0 .. 127)
// waves per block of k_actor (one block per CU: the block shares the LDS weight image).  The
// default-layout (DEF) forms fit more waves per SIMD: bf16 4 (<= 128 VGPRs), bf16x3 3 (<= 168); the
// generic forms and the fp32-faithful form (three operand planes) 2.
// (prec: the kernel's PREC — 1 bf16, 3 bf16x3, 4 the fp16-split fp32 form, 6 the three-way bf16 fp32 form)
constexpr int actor_max_waves(int prec, bool def) { return !def || prec == 6 ? 8 : prec == 1 ? 16 : 12; }
// the fp16-split form's per-layer weight scale: every scaled weight below 2^kActorF16Exp (k_actor_pack)
constexpr int kActorF16Exp = 0;
// ... and max |b1| s1 below 2^kActorF16Bias (layer 2's fp16 operand relu(layer 1) s1 stays in range)
constexpr int kActorF16Bias = 13;
// the packed tail: b1 [kActorRows] | b2 [kActorRows] | W3^T [kActorRows][kActorNA] | b3 [kActorNA] | s1
constexpr int kActorMaxU = 64;  // folded features (<= 8 own + 3 per message; <= 128 slots: <= 8 + 3 x 15)
constexpr int kActorTailS1 = (2 + kActorNA) * kActorRows + kActorNA;
constexpr int kActorTailFold = kActorTailS1 + 1;                  // ActorFold, 2 + 2 kActorMaxU ints
constexpr int kActorTailEnd = kActorTailFold + 2 + 2 * kActorMaxU;

// Shapes, the obs row's slot layout, byte offsets of the packed weight image (identical in global
// memory and in LDS) and of the per-block LDS work areas.  Filled by the host (mdr_capi.hip
// actor_layout).
//
// Slot layout: the K dimension of layer 1 is the obs row in 4-float chunks, [own features (n_own,
// zero padded to own4) | message 0 | ... | message K-1 (M each, zero padded to m4)]; the packed W1
// columns follow the same order.  LDS rows (per wave, stride rs floats, an odd multiple of 4):
//   ring:  one row per message source s (house b0 - lo + s): [message (m4) | own (own4)]
//   table: one row per tile house: [own (own4) | message 0 .. K-1 (m4 each)]
// The fp16-split form folds the house-independent features — own (obs_uniform_own: e.g. the cluster
// power P / R, ~0.4 N, beyond fp16 at 1M houses) and in messages (obs_uniform_msg: the hvac constants,
// e.g. a 15 kW capacity) — into its layer-1 bias once per block, in fp32 from the raw W1: their W1
// columns are packed as zero, and the own ones' row slots hold 0 (feat[0 .. nu_own)).  k_actor_pack
// writes the list into the packed tail after s1 (kActorTailFold: nu, nu_own, feat[64], cf[64] as ints),
// where k_actor reads it from LDS.
struct ActorFold {
  int nu, nu_own;
  int feat[kActorMaxU], cf[kActorMaxU];
  float cfmax[kActorMaxU];  // a bound on |cf| (the cluster power's: n_global max P_on / R; constants exact)
};
struct ActorDims {
  int n_in, h1, h2, n_act;
  int mb;         // row blocks of both hidden layers (ceil(max(h1, h2) / 16), 7 or 8)
  int ks1;        // layer-1 k-steps of 32: max(2, ceil(nslot / 32)) (the kernel's instantiations;
                  // a padding k-step reads zero weights and the zero chunk)
  int nf;         // fragments per (row block, k-step): 2 = (hi, lo), 3 = (hi, mid, lo) for the bf16 fp32 form
  int f16;        // 1: fp16 fragments (the fp16-split fp32 form, kernel PREC 4), scaled per layer
  const float* w1raw;  // the loaded fp32 W1 [h1][n_in] (the fp16-split form's folded features, ActorFold)
  int lds_b1;          // block LDS: that bias and b2, both times the launch's layer-1 scale, [2][kActorRows] floats
  int n_own, own4, msg_w, m4, n_comm, lo, ring, nslot, rs, nrows;
  int off_w1, off_w2, off_tail, off_end;  // packed image: W1 / W2 fragments, fp32 tail
  int lds_cf, lds_hist, lds_wave, wave_stride;  // block LDS: obs consts, count histogram, wave slices
  int w_zero, w_hw, w_cls;                       // offsets inside a wave slice (rows at 0)
  int lds_total;
};

struct ActorOut {
  uint8_t* action;               // [n] sampled action (u8), or null
  float* prob;                   // [n] probability of the sampled action, or null
  float* probs;                  // [n][n_act] all action probabilities, or null
  float* obs;                    // [n][n_in] the observation rows, or null
  unsigned long long* count_next;  // count slab of the tick these actions drive, or null
  unsigned long long* prof;        // diagnostics: [grid][8] per-phase shader cycles, or null
  int tiles;                       // 32-house tiles to run: 0 all, 1 interior (not the first or last), 2 the
                                   // first and last (the sharded ring halo's readers; mdr_actor_rollout_sharded)
  unsigned* ovf;                   // fp16-split form: [0] tiles that met a non-finite logit, [1] tiles whose
                                   // logits came from the scalar fp32 fallback (actor_tile_fp32), or null
};

__global__ void k_actor_pack(ActorDims d, ActorFold fo, const float* w1, const float* b1, const float* w2,
                             const float* b2, const float* w3, const float* b3, unsigned char* out);
template <int PREC, bool PROF, int MB, int KS1, bool DEF>
__global__ void k_actor(KParams p, ObsArgs o, ActorDims d, const double* p_dev,
                        const unsigned char* wpack, ActorOut out, uint64_t tick, const TickArgs* tkp);

// the general chain (mdr_actor.hip "chain"): one dense layer over fp32 rows, then the head
template <int PREC>
__global__ void k_dense(const float* X, int ldx, int K, int64_t n, const float* W, const float* b, int out, float* Y,
                        int ldy, int relu_on);
__global__ void k_actor_head(KParams p, const float* X, int ldx, int K, const float* W3, const float* b3,
                             uint64_t tick0, const TickArgs* tkp, ActorOut out);

}  // namespace mdr
