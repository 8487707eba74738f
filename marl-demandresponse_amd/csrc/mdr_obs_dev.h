// mdr_obs_dev.h — the norm_state_dict observation row (server/app/utils/norm.py:178-218) as
// device functions, shared by k_obs (obs tensor) and k_actor (obs fused with the MA-PPO actor).
//
// A block stages the message features of its ring neighbourhood once in LDS (obs_stage_ring),
// then every house's row is assembled from its own state + the staged messages (obs_build_row).
// Feature order and arithmetic follow norm.py exactly (float64 math, one cast to float32 per
// feature), so both kernels produce bit-identical rows.
#pragma once
#include "mdr_device.h"
#include "mdr_kernels.h"

namespace mdr {

// Message a house j sends (Building.message, building.py:101-139, normalised by
// norm.py:60-110): (T - target)/5, int(sso/L), P/R, P_max/R [, Ua, Ca, Cm, Hm ratios][, cop, lcf, cap]
__device__ __forceinline__ void msg_features(const KParams& p, const ObsArgs& o, int64_t j,
                                             float* dst) {
  const uint32_t w = p.hvac[j];
  const int cls = p.cap_idx[j];
  const double pmax = p.p_on[cls];
  const double R = o.norm_reg_sig;
  dst[0] = (float)((p.t_air[j] - p.target[j]) / 5.0);
  dst[1] = (float)trunc((double)hv_sso(w) / (double)p.L);
  dst[2] = (float)((hv_on(w) ? pmax : 0.0) / R);
  dst[3] = (float)(pmax / R);
  int f = 4;
  if (o.msg_thermal) {
    dst[f++] = (float)(p.ua[j] / o.cfg_ua);
    dst[f++] = (float)(p.ca[j] / o.cfg_ca);
    dst[f++] = (float)(p.cm[j] / o.cfg_cm);
    dst[f++] = (float)(p.hm[j] / o.cfg_hm);
  }
  if (o.msg_hvac) {
    dst[f++] = (float)o.cfg_cop;
    dst[f++] = (float)o.cfg_lcf;
    dst[f++] = (float)o.cfg_cap;
  }
}

// RING topology: message sources of the houses [b0, b0 + nb) are [b0 - lo, b0 + nb + hi);
// their features go to msg[(s) * M] for s = 0 .. lo + nb + hi.  Threads tid, tid + nthr, ...
__device__ __forceinline__ void obs_stage_ring(const KParams& p, const ObsArgs& o, int64_t b0, int nb,
                                               float* msg, int tid, int nthr) {
  const int K = o.n_comm, M = o.msg_w;
  if (o.comm_mode != MDR_COMM_RING || K <= 0) return;
  const int lo = K / 2, hi = (K + 1) / 2;
  const int nsrc = lo + nb + hi;
  for (int s = tid; s < nsrc; s += nthr) {
    int64_t j = b0 - lo + s;  // local index, may fall outside the shard
    if (o.halo_msg && (j < 0 || j >= p.n)) {
      // multi-GPU ring: [0, lo) = houses before the shard, [lo, lo+hi) = houses after it
      const int h = j < 0 ? (int)(j + lo) : (int)(lo + (j - p.n));
      for (int m = 0; m < M; ++m) msg[s * M + m] = o.halo_msg[h * M + m];
    } else {
      j %= p.n;
      if (j < 0) j += p.n;
      msg_features(p, o, j, msg + s * M);
    }
  }
}

// The F-wide row of local house i (= b0 + t) into row[0 .. F).  P: cluster power of the tick.
// The hvac word is returned (callers that need the FSM state reuse the load).
__device__ __forceinline__ uint32_t obs_build_row(const KParams& p, const ObsArgs& o, double P,
                                                  int64_t i, int t, const float* msg, float* row) {
  const int M = o.msg_w, K = o.n_comm;
  const int lo = K / 2;
  const double R = o.norm_reg_sig;
  const uint32_t w = p.hvac[i];
  int f = 0;
  row[f++] = hv_on(w) ? 1.f : 0.f;
  row[f++] = hv_lock(w) ? 1.f : 0.f;
  row[f++] = (float)trunc((double)hv_sso(w) / (double)p.L);
  row[f++] = 1.f;  // int(lockout_duration / lockout_duration)
  if (o.hvac_state) { row[f++] = (float)(o.cfg_cop / o.cfg_cop); row[f++] = (float)(o.cfg_lcf / o.cfg_lcf); }
  row[f++] = (float)(P / R);
  row[f++] = (float)(o.s / (R * (double)p.n_global));
  row[f++] = (float)p.deadband;
  const double tgt = p.target[i];
  row[f++] = (float)((p.t_air[i] - 20.0) / 5.0);
  row[f++] = (float)((p.t_mass[i] - 20.0) / 5.0);
  row[f++] = (float)((tgt - 20.0) / 5.0);
  if (o.solar_state) row[f++] = (float)(o.solar / 1000.0);
  if (o.thermal_state) {
    row[f++] = (float)(p.ua[i] / o.cfg_ua);
    row[f++] = (float)(p.ca[i] / o.cfg_ca);
    row[f++] = (float)(p.cm[i] / o.cfg_cm);
    row[f++] = (float)(p.hm[i] / o.cfg_hm);
    row[f++] = (float)((o.t_od - 20.0) / 5.0);
  }
  if (K > 0) {
    if (o.comm_mode == MDR_COMM_RING) {
      // neighbours [i-lo .. i-1, i+1 .. i+hi] (agent_communication_builder.py:65-83)
      for (int k = 0; k < K; ++k) {
        const int s = k < lo ? (t + k) : (t + lo + 1 + (k - lo));
        for (int m = 0; m < M; ++m) row[f++] = msg[s * M + m];
      }
    } else {
      float tmp[16];
      for (int k = 0; k < K; ++k) {
        const int64_t j = o.comm_table[i * K + k];
        msg_features(p, o, j, tmp);
        for (int m = 0; m < M; ++m) row[f++] = tmp[m];
      }
    }
  }
  return w;
}

}  // namespace mdr
