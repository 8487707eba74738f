// mdr_obs_dev.h — the norm_state_dict observation row (server/app/utils/norm.py:178-218) as
// device functions, shared by k_obs (obs tensor) and k_actor (obs fused with the MA-PPO actor).
//
// A house's state is loaded once into registers (HouseRegs); its message features
// (msg_from_regs) and its own row features (row_scalars) are computed from them.  Feature order
// and arithmetic follow norm.py exactly (float64 math, one cast to float32 per feature), so every
// kernel that uses these functions produces bit-identical rows.
#pragma once
#include "mdr_device.h"
#include "mdr_kernels.h"

namespace mdr {

struct HouseRegs {
  double T, Tm, tg, ua, ca, cm, hm;
  uint32_t w;
  int cls;
};

// thermal: also load Ua, Ca, Cm, Hm (state_prop.thermal / message_prop.thermal)
__device__ __forceinline__ void house_load(const KParams& p, int64_t j, bool thermal, HouseRegs& r) {
  r.T = p.t_air[j];
  r.Tm = p.t_mass[j];
  r.tg = p.target[j];
  r.w = p.hvac[j];
  r.cls = p.cap_idx[j];
  if (thermal) {
    r.ua = p.ua[j];
    r.ca = p.ca[j];
    r.cm = p.cm[j];
    r.hm = p.hm[j];
  } else {
    r.ua = r.ca = r.cm = r.hm = 0.0;
  }
}

__device__ __forceinline__ bool obs_needs_thermal(const ObsArgs& o) { return o.thermal_state || o.msg_thermal; }

// House-independent features of a tick, computed once per block into LDS (float32, each from the
// same float64 expression norm.py evaluates):
//   cf[0] int(L / L) = 1, cf[1] cop/cop, cf[2] lcf/lcf, cf[3] P/R, cf[4] S/(R N), cf[5] deadband,
//   cf[6] solar/1000, cf[7] (T_od - 20)/5, cf[8..10] message hvac constants (cop, lcf, cap),
//   cf[kObsPmr + k] P_max(class k)/R  (a message's curr/max consumption features).
constexpr int kObsPmr = 16;
constexpr int kObsConst = kObsPmr + MDR_MAX_CAP;
__device__ __forceinline__ void obs_consts(const KParams& p, const ObsArgs& o, double P, float* cf, int tid,
                                           int nthr) {
  const double R = o.norm_reg_sig;
  if (tid == 0) {
    cf[0] = 1.f;
    cf[1] = (float)(o.cfg_cop / o.cfg_cop);
    cf[2] = (float)(o.cfg_lcf / o.cfg_lcf);
    cf[3] = (float)(P / R);
    cf[4] = (float)(o.s / (R * (double)p.n_global));
    cf[5] = (float)p.deadband;
    cf[6] = (float)(o.solar / 1000.0);
    cf[7] = (float)((o.t_od - 20.0) / 5.0);
    cf[8] = (float)o.cfg_cop;
    cf[9] = (float)o.cfg_lcf;
    cf[10] = (float)o.cfg_cap;
  }
  for (int k = tid; k < p.n_cap; k += nthr) cf[kObsPmr + k] = (float)(p.p_on[k] / R);
}

// The divisions of the row expressions, set up once per kernel: x / 5.0 as the shared-reciprocal
// sequence (mdr_device.h Recip: bit-identical to the IEEE quotient; the operator for zero,
// non-finite or extreme x), and int(sso / L) as a multiply by the float64 reciprocal of L with one
// correction (for sso < 2^30 the product is within 2^-52 relative of sso / L, so its truncation is
// the quotient or one less; exact multiples are corrected up).
struct ObsDiv {
  Recip r5;
  double rL;
  uint32_t L;
};
__device__ __forceinline__ ObsDiv obs_div(const KParams& p) {
  ObsDiv d;
  d.r5 = recip(5.0);
  d.L = p.L < 1 ? 1u : (uint32_t)p.L;
  d.rL = 1.0 / (double)d.L;
  return d;
}
__device__ __forceinline__ double div5(double a, const ObsDiv& dv) {
  return div_safe(a) ? div_by(a, dv.r5) : a / 5.0;
}
// int(sso / L) of norm.py (sso < 2^30: the float64 quotient never rounds up to the next integer,
// so truncating it equals the integer quotient)
__device__ __forceinline__ float sso_ratio(uint32_t w, const ObsDiv& dv) {
  const uint32_t a = hv_sso(w);
  uint32_t q = (uint32_t)((double)a * dv.rL);
  q += a - q * dv.L >= dv.L ? 1u : 0u;
  return (float)q;
}

// Message a house sends (Building.message, building.py:101-139, normalised by norm.py:60-110):
// (T - target)/5, int(sso/L), P/R, P_max/R [, Ua, Ca, Cm, Hm ratios][, cop, lcf, cap]
__device__ __forceinline__ void msg_from_regs(const KParams& p, const ObsArgs& o, const HouseRegs& r,
                                              const float* cf, float* dst, const ObsDiv& dv) {
  const float pmr = cf[kObsPmr + r.cls];
  dst[0] = (float)div5(r.T - r.tg, dv);
  dst[1] = sso_ratio(r.w, dv);
  dst[2] = hv_on(r.w) ? pmr : 0.f;  // (0.0 / R) == +0
  dst[3] = pmr;
  int f = 4;
  if (o.msg_thermal) {
    dst[f++] = (float)(r.ua / o.cfg_ua);
    dst[f++] = (float)(r.ca / o.cfg_ca);
    dst[f++] = (float)(r.cm / o.cfg_cm);
    dst[f++] = (float)(r.hm / o.cfg_hm);
  }
  if (o.msg_hvac) {
    dst[f++] = cf[8];
    dst[f++] = cf[9];
    dst[f++] = cf[10];
  }
}

// The house-independent features of a message in msg_from_regs' order (the hvac constants cf[8..10]):
// off[u] = the offset inside the message, cfk[u] = the obs_consts entry; returns how many (<= 3).
// Keep in step with msg_from_regs.
__host__ __device__ inline int obs_uniform_msg(int msg_thermal, int msg_hvac, int* off, int* cfk) {
  if (!msg_hvac) return 0;
  const int f = 4 + (msg_thermal ? 4 : 0);
  for (int u = 0; u < 3; ++u) { off[u] = f + u; cfk[u] = 8 + u; }
  return 3;
}

__device__ __forceinline__ void msg_features(const KParams& p, const ObsArgs& o, int64_t j, const float* cf,
                                             float* dst, const ObsDiv& dv) {
  HouseRegs r;
  house_load(p, j, o.msg_thermal != 0, r);
  msg_from_regs(p, o, r, cf, dst, dv);
}

// The house's own features (everything before the messages); returns how many were written.
// zu: the house-independent ones (the cf[k] entries, obs_uniform_own) written as 0 — the fp16-split
// actor adds their contribution to its layer-1 bias once per block instead (mdr_actor.hip)
__device__ __forceinline__ int row_scalars(const KParams& p, const ObsArgs& o, const HouseRegs& r,
                                           const float* cf, float* row, const ObsDiv& dv, bool zu = false) {
  int f = 0;
  row[f++] = hv_on(r.w) ? 1.f : 0.f;
  row[f++] = hv_lock(r.w) ? 1.f : 0.f;
  row[f++] = sso_ratio(r.w, dv);
  row[f++] = zu ? 0.f : cf[0];
  if (o.hvac_state) { row[f++] = zu ? 0.f : cf[1]; row[f++] = zu ? 0.f : cf[2]; }
  row[f++] = zu ? 0.f : cf[3];
  row[f++] = zu ? 0.f : cf[4];
  row[f++] = zu ? 0.f : cf[5];
  row[f++] = (float)div5(r.T - 20.0, dv);
  row[f++] = (float)div5(r.Tm - 20.0, dv);
  row[f++] = (float)div5(r.tg - 20.0, dv);
  if (o.solar_state) row[f++] = zu ? 0.f : cf[6];
  if (o.thermal_state) {
    row[f++] = (float)(r.ua / o.cfg_ua);
    row[f++] = (float)(r.ca / o.cfg_ca);
    row[f++] = (float)(r.cm / o.cfg_cm);
    row[f++] = (float)(r.hm / o.cfg_hm);
    row[f++] = zu ? 0.f : cf[7];
  }
  return f;
}

// The house-independent own features of row_scalars' order: feat[u] = the feature index, cfk[u] = the
// obs_consts entry it holds; returns how many (<= kObsUniformMax).  Keep in step with row_scalars.
constexpr int kObsUniformMax = 8;
__host__ __device__ inline int obs_uniform_own(int hvac_state, int solar_state, int thermal_state, int* feat,
                                               int* cfk) {
  int f = 3, u = 0;  // (on, lock, sso ratio first)
  feat[u] = f++; cfk[u++] = 0;
  if (hvac_state) { feat[u] = f++; cfk[u++] = 1; feat[u] = f++; cfk[u++] = 2; }
  feat[u] = f++; cfk[u++] = 3;
  feat[u] = f++; cfk[u++] = 4;
  feat[u] = f++; cfk[u++] = 5;
  f += 3;  // (T, Tm, target)
  if (solar_state) { feat[u] = f++; cfk[u++] = 6; }
  if (thermal_state) { f += 4; feat[u] = f++; cfk[u++] = 7; }
  return u;
}

// RING topology: message sources of the houses [b0, b0 + nb) are [b0 - lo, b0 + nb + hi);
// their features go to msg[(s) * M] for s = 0 .. lo + nb + hi.  Threads tid, tid + nthr, ...
__device__ __forceinline__ void obs_stage_ring(const KParams& p, const ObsArgs& o, int64_t b0, int nb,
                                               const float* cf, float* msg, int tid, int nthr, const ObsDiv& dv) {
  const int K = o.n_comm, M = o.msg_w;
  if (o.comm_mode != MDR_COMM_RING || K <= 0) return;
  const int lo = K / 2, hi = (K + 1) / 2;
  const int nsrc = lo + nb + hi;
  for (int s = tid; s < nsrc; s += nthr) {
    int64_t j = b0 - lo + s;  // local index, may fall outside the shard
    if (o.halo_msg && (j < 0 || j >= p.n)) {
      // multi-GPU ring: [0, lo) = houses before the shard, [lo, lo+hi) = houses after it
      const int h = j < 0 ? (int)(j + lo) : (int)(lo + (j - p.n));
      const float* src = o.halo_next && h >= lo ? o.halo_next + (size_t)(h - lo) * M : o.halo_msg + (size_t)h * M;
      for (int m = 0; m < M; ++m) msg[s * M + m] = src[m];
    } else {
      j %= p.n;
      if (j < 0) j += p.n;
      msg_features(p, o, j, cf, msg + s * M, dv);
    }
  }
}

// Messages of local house i (row index t in the block tile) appended at row[f ..).
__device__ __forceinline__ void row_messages(const KParams& p, const ObsArgs& o, int64_t i, int t,
                                             const float* cf, const float* msg, float* row, int f,
                                             const ObsDiv& dv) {
  const int M = o.msg_w, K = o.n_comm;
  const int lo = K / 2;
  if (K <= 0) return;
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
      if (o.msg_all) {  // sharded: the all-gathered rows, global ids
        for (int m = 0; m < M; ++m) row[f++] = o.msg_all[j * M + m];
        continue;
      }
      msg_features(p, o, j, cf, tmp, dv);
      for (int m = 0; m < M; ++m) row[f++] = tmp[m];
    }
  }
}

// The F-wide row of local house i (= b0 + t) into row[0 .. F); cf: obs_consts of the tick.
// The hvac word is returned (callers that need the FSM state reuse the load).
__device__ __forceinline__ uint32_t obs_build_row(const KParams& p, const ObsArgs& o, int64_t i, int t,
                                                  const float* cf, const float* msg, float* row,
                                                  const ObsDiv& dv) {
  HouseRegs r;
  house_load(p, i, o.thermal_state != 0, r);
  const int f = row_scalars(p, o, r, cf, row, dv);
  row_messages(p, o, i, t, cf, msg, row, f, dv);
  return r.w;
}

}  // namespace mdr
