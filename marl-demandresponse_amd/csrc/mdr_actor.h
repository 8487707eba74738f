// mdr_actor.h — parameter blocks of the fused obs + MA-PPO actor kernels (mdr_actor.hip).
#pragma once
#include "mdr_kernels.h"

namespace mdr {

constexpr int kActorMB = 4;       // 32-row MFMA blocks per hidden layer (hidden width <= 128)
constexpr int kActorRows = 32 * kActorMB;
constexpr int kActorNA = 2;       // actions: on / off (MAPPO num_action = 2, mappo.py:38)
constexpr int kActorMaxIn = 128;  // obs features (8 k-steps of 16)

// Shapes + byte offsets of the packed weight image (identical in global memory and in LDS) and
// of the per-block LDS work areas.  Filled by the host (mdr_capi.hip actor_layout).
struct ActorDims {
  int n_in, h1, h2, n_act;
  int ks1, ks2;  // k-steps of layer 1 (ceil(n_in/16)) and layer 2 (ceil(h1/16))
  int fs;        // LDS obs row stride (floats): >= n_in, multiple of 4, odd multiple of 4 words
  int nf;        // bf16 fragments per (row block, k-step): 2 = (hi, lo), 3 = (hi, mid, lo) for MDR_PREC_FP32
  int off_w1, off_w2, off_tail, off_end;  // packed image: W1 / W2 fragments, fp32 tail
  int lds_cf, lds_hist, lds_wave, wave_stride;  // block LDS: obs consts, count histogram, wave slices
  int w_msg, w_hw, w_cls;                        // offsets inside a wave slice (rows at 0)
  int lds_total;
};

struct ActorOut {
  uint8_t* action;               // [n] sampled action (u8), or null
  float* prob;                   // [n] probability of the sampled action, or null
  float* probs;                  // [n][n_act] all action probabilities, or null
  float* obs;                    // [n][n_in] the observation rows, or null
  unsigned long long* count_next;  // count slab of the tick these actions drive, or null
  unsigned long long* prof;        // diagnostics: [grid][8] per-phase shader cycles, or null
};

__global__ void k_actor_pack(ActorDims d, const float* w1, const float* b1, const float* w2,
                             const float* b2, const float* w3, const float* b3, unsigned char* out);
template <int PREC, bool PROF>
__global__ void k_actor(KParams p, ObsArgs o, ActorDims d, const double* p_dev,
                        const unsigned char* wpack, ActorOut out, uint64_t tick, const TickArgs* tkp);

}  // namespace mdr
