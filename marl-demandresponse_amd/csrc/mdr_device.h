// mdr_device.h — per-house device math for the vectorised environment step (gfx950).
//
// Every floating-point expression keeps the reference's operation order (Python evaluates
// left to right, one IEEE-754 rounding per operation); the library is compiled with
// -ffp-contract=off so no a*b+c is fused into an FMA.  Division and sqrt are correctly rounded
// on gfx950 (v_div_scale/v_div_fmas/v_div_fixup; v_sqrt_f64 + refinement), exp is ocml's
// (<= 1 ulp), so a tick agrees with the reference to ~1e-13 relative and integer state is
// bit-exact.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mdr {

constexpr uint32_t kOnBit = 1u << 31;
constexpr uint32_t kLockBit = 1u << 30;
constexpr uint32_t kSsoMask = (1u << 30) - 1u;  // seconds_since_off saturates at 2^30-1 s (34 y)

// ---------------------------------------------------------------------------- lockout FSM
// HVAC.step, server/app/core/environment/cluster/hvac.py:43-64:
//   if not on: sso += dt
//   lockout = not (on or sso >= L)
//   if lockout: on = False
//   else: on = action; if on: sso = 0 elif sso + dt < L: lockout = True
// 32-bit arithmetic: sso <= 2^30 - 1 and 0 <= dt < 2^31 (mdr_create rejects dt < 0), so
// sso + dt < 2^32 never wraps; a negative L behaves as 0 (sso >= L always, sso + dt < L never).
__device__ __forceinline__ uint32_t hvac_fsm(uint32_t w, bool action, int dt, int L) {
  const bool on = (w & kOnBit) != 0;
  const uint32_t Lu = L < 0 ? 0u : (uint32_t)L;
  uint32_t sso = w & kSsoMask;
  if (!on) sso += (uint32_t)dt;
  const bool locked = !(on || sso >= Lu);
  bool non = false, nlock = locked;
  if (!locked) {
    non = action;
    if (non) sso = 0;
    else if (sso + (uint32_t)dt < Lu) nlock = true;
  }
  sso = sso < kSsoMask ? sso : kSsoMask;
  return sso | (nlock ? kLockBit : 0u) | (non ? kOnBit : 0u);
}

__device__ __forceinline__ bool hv_on(uint32_t w) { return (w & kOnBit) != 0; }
__device__ __forceinline__ bool hv_lock(uint32_t w) { return (w & kLockBit) != 0; }
__device__ __forceinline__ uint32_t hv_sso(uint32_t w) { return w & kSsoMask; }

// ---------------------------------------------------------------------------- RC thermal
// Building.update_temperature, server/app/core/environment/cluster/building.py:141-222
// (GridLAB-D 2-node analytic solution), split into the part that depends only on the house's
// parameters (rc_coeffs: roots r1, r2 of the characteristic polynomial, mass/air ratios A3, A4
// and the decay factors exp(r dt)) and the per-tick part (rc_apply).  Both keep the reference's
// operation order, so a cached RcCoef gives bit-identical results to recomputing it every tick.
// q_hvac = HVAC.get_heat_transfer (hvac.py:85-99), solar = compute_solar_gain (per-tick scalar),
// t_od = previous tick's outdoor temperature.
// ---------------------------------------------------------------------------- exact division
// a / b correctly rounded with the reciprocal shared by every quotient that has the same
// divisor.  This is the gfx950 IEEE division sequence LLVM emits for fdiv f64 (v_rcp_f64, two
// Newton steps, q0 = a*y, r = fma(-b, q0, a), q = fma(r, y, q0); Markstein's theorem makes the
// final correction exact) minus v_div_scale / v_div_fixup, which only act for denormals, zero /
// inf / nan operands or operand exponents 768+ apart.  Callers check `Recip::safe` (divisor and
// numerators within [2^-300, 2^300]) and fall back to the plain operator otherwise, so results
// are bit-identical to `a / b` (tests/test_division_gpu.py checks this on 10^8 random pairs).
struct Recip {
  double b, nb, y;
};

__device__ __forceinline__ Recip recip(double b) {
  Recip r;
  r.b = b;
  r.nb = -b;
  double y = __builtin_amdgcn_rcp(b);
  const double e0 = __builtin_fma(r.nb, y, 1.0);
  y = __builtin_fma(y, e0, y);
  const double e1 = __builtin_fma(r.nb, y, 1.0);
  r.y = __builtin_fma(y, e1, y);
  return r;
}

__device__ __forceinline__ double div_by(double a, const Recip& r) {
  const double q0 = a * r.y;
  const double rem = __builtin_fma(r.nb, q0, a);
  return __builtin_fma(rem, r.y, q0);
}

// |x| in [2^-300, 2^300] (zero excluded): no scaling can trigger in the hardware sequence
__device__ __forceinline__ bool div_safe(double x) {
  const uint32_t e = (uint32_t)(__double_as_longlong(x) >> 52) & 0x7FF;
  return e >= 1023 - 300 && e <= 1023 + 300;
}

// ---------------------------------------------------------------------------- RC coefficients
struct RcCoef { double r1, r2, A3, A4, e1, e2; };

// FAST = shared-reciprocal division (callers guarantee div_safe operands)
template <bool FAST>
__device__ __forceinline__ RcCoef rc_coeffs_t(double Ua, double Ca, double Cm, double Hm, double dt) {
  RcCoef k;
  const double UaHm = Ua + Hm;
  const double c = Ua;
  double a, b, UaHm_Hm, r1Ca_Hm, r2Ca_Hm;
  if (FAST) {
    const Recip rH = recip(Hm);
    a = div_by(Cm * Ca, rH);
    b = div_by(Cm * UaHm, rH) + Ca;
    const double disc = __builtin_sqrt(b * b - 4.0 * a * c);
    const Recip r2a = recip(2.0 * a);
    k.r1 = div_by(-b + disc, r2a);
    k.r2 = div_by(-b - disc, r2a);
    UaHm_Hm = div_by(UaHm, rH);
    r1Ca_Hm = div_by(k.r1 * Ca, rH);
    r2Ca_Hm = div_by(k.r2 * Ca, rH);
  } else {
    a = Cm * Ca / Hm;
    b = Cm * UaHm / Hm + Ca;
    const double disc = __builtin_sqrt(b * b - 4.0 * a * c);
    const double two_a = 2.0 * a;
    k.r1 = (-b + disc) / two_a;
    k.r2 = (-b - disc) / two_a;
    UaHm_Hm = UaHm / Hm;
    r1Ca_Hm = k.r1 * Ca / Hm;
    r2Ca_Hm = k.r2 * Ca / Hm;
  }
  k.A3 = r1Ca_Hm + UaHm_Hm;
  k.A4 = r2Ca_Hm + UaHm_Hm;
  k.e1 = exp(k.r1 * dt);
  k.e2 = exp(k.r2 * dt);
  return k;
}

__device__ __forceinline__ RcCoef rc_coeffs(double Ua, double Ca, double Cm, double Hm, double dt) {
  return rc_coeffs_t<false>(Ua, Ca, Cm, Hm, dt);
}

template <bool FAST>
__device__ __forceinline__ void rc_apply_t(double T, double Tm, double Ua, double Ca, double Hm,
                                           const RcCoef& k, double q_hvac, double solar, double t_od,
                                           double& T_out, double& Tm_out) {
  const double od_k = t_od + 273.0;
  const double t_k = T + 273.0;
  const double tm_k = Tm + 273.0;
  const double Qa = q_hvac + solar;
  const double UaHm = Ua + Hm;
  const double c = Ua;
  const double d = Qa + Ua * od_k;  // Qm (= 0) + Qa + Ua * od_k
  double dTA0dt, d_c, r2d_c, A1;
  if (FAST) {
    const Recip rCa = recip(Ca);
    const Recip rc = recip(c);
    dTA0dt = div_by(Hm * tm_k, rCa) - div_by(UaHm * t_k, rCa) + div_by(Ua * od_k, rCa) + div_by(Qa, rCa);
    d_c = div_by(d, rc);
    r2d_c = div_by(k.r2 * d, rc);
    A1 = div_by(k.r2 * t_k - dTA0dt - r2d_c, recip(k.r2 - k.r1));
  } else {
    dTA0dt = Hm * tm_k / Ca - UaHm * t_k / Ca + Ua * od_k / Ca + Qa / Ca;
    d_c = d / c;
    r2d_c = k.r2 * d / c;
    A1 = (k.r2 * t_k - dTA0dt - r2d_c) / (k.r2 - k.r1);
  }
  const double A2 = t_k - d_c - A1;
  const double t_new = A1 * k.e1 + A2 * k.e2 + d_c;
  // the reference adds g (= Qm/Hm = 0.0) before d/c; x + 0.0 differs from x only for x = -0.0, and
  // then only in the sign of a zero tm_new, which the "- 273" below maps to the same -273.0: the
  // addition cannot change T_mass, so it is not evaluated
  const double tm_new = A1 * k.A3 * k.e1 + A2 * k.A4 * k.e2 + d_c;
  T_out = t_new - 273.0;
  Tm_out = tm_new - 273.0;
}

// deadbandL2 with deadband = 0 (the default): hi = lo = target + 0.0, and both branches of the
// reference give (value - target)^2; value == target or NaN gives 0.0 — branch-free
__device__ __forceinline__ double deadband_l2_0(double hi, double value) {
  const double x = value - hi;
  return (value < hi || value > hi) ? x * x : 0.0;
}

// deadbandL2, server/app/utils/utils.py:4-23  (x**2 evaluated as x*x)
__device__ __forceinline__ double deadband_l2(double target, double deadband, double value) {
  const double hi = target + deadband / 2.0;
  const double lo = target - deadband / 2.0;
  if (hi < value) { const double x = value - hi; return x * x; }
  if (lo > value) { const double x = lo - value; return x * x; }
  return 0.0;
}

// ---------------------------------------------------------------------------- controllers
// BangBangController.act (bangbang_controllers.py:54-65): on iff T > target.
__device__ __forceinline__ bool ctrl_bangbang(double T, double target) { return T > target; }
// DeadbandBangBangController.act (bangbang_controllers.py:25-42).
__device__ __forceinline__ bool ctrl_deadband(double T, double target, double deadband, bool on) {
  if (T < target - deadband / 2.0) return false;
  if (T > target + deadband / 2.0) return true;
  return on;
}

// ---------------------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Random controller: Bernoulli(0.5) per (house, tick).  The bit of global house gid at tick t is
// bit (gid & 63) of the first 64 bits of Philox4x32-10(seed; counter = (gid >> 6, t)), so it does
// not depend on sharding or on how houses map to threads.  One wave evaluates the generator ONCE
// for all its houses and both ticks it needs (t and t + 1): lanes 0..31 take the 64-house groups
// starting at the wave's first id for tick t, lanes 32..63 the same groups for t + 1, and every
// house fetches its word from the owning lane (4 cross-lane reads).  All lanes of the wave must
// call it with the same wave-uniform gbase (first id of the wave) and tick; a wave may span at
// most 32 groups (here <= 3).
__device__ __forceinline__ void philox_words(uint64_t seed, uint64_t grp, uint64_t t, uint32_t& lo,
                                             uint32_t& hi) {
  const u32x4 r = philox4x32_10(u32x4{(uint32_t)grp, (uint32_t)(grp >> 32), (uint32_t)t,
                                      (uint32_t)(t >> 32) ^ 0x5A17u},
                                (uint32_t)seed, (uint32_t)(seed >> 32));
  lo = r.x;
  hi = r.y;
}

__device__ __forceinline__ bool bit_of(uint32_t lo, uint32_t hi, uint64_t gid) {
  const int b = (int)(gid & 63);
  return ((b < 32 ? (lo >> b) : (hi >> (b - 32))) & 1u) != 0;
}

struct WaveRandom {
  uint32_t lo, hi;  // this lane's generator words
  uint64_t g0;      // first 64-house group of the wave
  __device__ __forceinline__ WaveRandom(uint64_t seed, uint64_t gbase, uint64_t t) {
    const int lane = threadIdx.x & 63;
    g0 = gbase >> 6;
    philox_words(seed, g0 + (lane & 31), t + (lane >> 5), lo, hi);
  }
  // action of house gid at tick t (next = false) or t + 1 (next = true)
  __device__ __forceinline__ bool get(uint64_t gid, bool next) const {
    const int src = (int)((gid >> 6) - g0) + (next ? 32 : 0);
    return bit_of((uint32_t)__shfl((int)lo, src), (uint32_t)__shfl((int)hi, src), gid);
  }
};

__device__ __forceinline__ double u01(uint32_t x) { return ((double)x + 0.5) * 2.3283064365386963e-10; }

}  // namespace mdr
