// mdr_interp.hip — interpolated base power.
//
// PowerInterpolator.interpolate_power (server/app/core/environment/power_grid/interpolation.py:186-243)
// for the houses the host sampled (random.choices, part of the reference's RNG contract), read
// straight from the device state:
//   * clip_interpolation_point (:245-264) on every axis;
//   * nearest grid point on the Ua/Cm/Ca/Hm-ratio axes (:152-162) and the HVAC_power axis
//     (:164-167): np.argmin of |grid - x|, the first minimum;
//   * multilinear interpolation over air_temp, mass_temp, OD_temp, hour, date (:169-176, scipy
//     interpn "linear" = RegularGridInterpolator._evaluate_linear): interval i = the largest with
//     grid[i] <= x (at most len-2), y = (x - grid[i]) / (grid[i+1] - grid[i]); the 32 corners in
//     itertools.product order (last axis fastest, (i, 1-y) before (i+1, y)), weight = ((((1*w0)*w1)
//     *w2)*w3)*w4, value = value + table[corner] * weight.
// Built with -ffp-contract=off, so each value is the reference's bit for bit; k_interp_sum adds the
// values in sample order (the reference's Python loop) and scales by N / k.
#include "mdr_interp.h"

namespace mdr {

__global__ void __launch_bounds__(64) k_interp_values(KParams p, InterpArgs d, const int64_t* __restrict__ ids,
                                                      int n, double od, double hour, double date,
                                                      double* __restrict__ vals) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int64_t j = ids[s] - p.goff;
  if (j < 0 || j >= p.n) {  // another shard's house: its owner writes the value (sum-allreduce)
    vals[s] = 0.0;
    return;
  }
  const double tg = p.target[j];
  // the point in dict_keys order (interpolation.py:226-237)
  double x[kInterpAxes];
  x[0] = p.ua[j] / d.cfg[0];
  x[1] = p.cm[j] / d.cfg[1];
  x[2] = p.ca[j] / d.cfg[2];
  x[3] = p.hm[j] / d.cfg[3];
  x[4] = p.t_air[j] - tg;
  x[5] = p.t_mass[j] - tg;
  x[6] = od - tg;
  x[7] = d.cap[p.cap_idx[j]];
  x[8] = hour;
  x[9] = date;
  int64_t base = 0;
  int idx[kInterpLinear];
  double y[kInterpLinear];
#pragma unroll
  for (int a = 0, q = 0; a < kInterpAxes; ++a) {
    double v = x[a];
    if (v > d.hi[a]) v = d.hi[a];
    else if (v < d.lo[a]) v = d.lo[a];
    const double* g = d.grid + d.off[a];
    const int len = d.len[a];
    if (a < 4 || a == 7) {
      int best = 0;
      double bd = fabs(g[0] - v);
      for (int k = 1; k < len; ++k) {
        const double e = fabs(g[k] - v);
        if (e < bd) { bd = e; best = k; }
      }
      base += (int64_t)best * d.stride[a];
    } else {
      int i = 0;
      while (i + 2 < len && g[i + 1] <= v) ++i;
      idx[q] = i;
      y[q] = (v - g[i]) / (g[i + 1] - g[i]);
      ++q;
    }
  }
  double value = 0.0;
  for (int c = 0; c < (1 << kInterpLinear); ++c) {
    double w = 1.0;
    int64_t o = base;
#pragma unroll
    for (int k = 0; k < kInterpLinear; ++k) {
      const int b = (c >> (kInterpLinear - 1 - k)) & 1;
      w = w * (b ? y[k] : 1.0 - y[k]);
      o += (int64_t)(idx[k] + b) * d.lstride[k];
    }
    value = value + d.table[o] * w;
  }
  vals[s] = value;
}

// base_power = 0.0; base_power += v (sample order); base_power *= multi_factor (interpolation.py:202-241)
__global__ void k_interp_sum(const double* __restrict__ vals, int n, double factor, double* out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  double b = 0.0;
  for (int s = 0; s < n; ++s) b = b + vals[s];
  out[0] = b * factor;
}

}  // namespace mdr
