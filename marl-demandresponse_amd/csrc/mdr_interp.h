// mdr_interp.h — interpolated base power: kernel arguments.
#pragma once
#include "mdr_kernels.h"

namespace mdr {

constexpr int kInterpAxes = MDR_INTERP_AXES;  // dict_keys order (interp_dict_keys.csv)
constexpr int kInterpLinear = 5;               // air_temp, mass_temp, OD_temp, hour, date

// Everything k_interp_values needs, by value.  Axes 0-3 (Ua/Cm/Ca/Hm ratios) and 7 (HVAC_power)
// are nearest-point axes, 4, 5, 6, 8, 9 multilinear ones (interpolation.py:147-176).
struct InterpArgs {
  const double* grid;   // concatenated axis values, axis a at grid[off[a] .. off[a] + len[a])
  const double* table;  // C order over the axes
  const double* cap;    // cooling capacity of each capacity class (HVAC_power of a house)
  double cfg[4];        // default_building_props Ua, Cm, Ca, Hm (the ratio denominators)
  double lo[kInterpAxes], hi[kInterpAxes];  // clip bounds: np.min / np.max of the axis values
  int64_t stride[kInterpAxes];
  int64_t lstride[kInterpLinear];           // strides of the linear axes, in corner order
  int off[kInterpAxes], len[kInterpAxes];
};

__global__ void k_interp_values(KParams p, InterpArgs d, const int64_t* ids, int n, double od, double hour,
                                double date, double* vals);
__global__ void k_interp_sum(const double* vals, int n, double factor, double* out);

}  // namespace mdr
