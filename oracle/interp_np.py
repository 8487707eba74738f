"""ORACLE (test infrastructure only): CPU restatement of the interpolated base power.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg use this module;
the product path (mdr_amd + libmdr_hip) never imports it.

Reference (file:line under /root/reference):
  PowerInterpolator.__init__            server/app/core/environment/power_grid/interpolation.py:50-91
  interpolate_grid_fast                 server/app/core/environment/power_grid/interpolation.py:137-178
  interpolate_power (sampling, sum)     server/app/core/environment/power_grid/interpolation.py:186-243
  clip_interpolation_point              server/app/core/environment/power_grid/interpolation.py:245-264
  PowerGrid.power_step (update period)  server/app/core/environment/power_grid/power_grid.py:60-66,149-161

The multilinear part is scipy's ``interpn(method="linear")`` (RegularGridInterpolator,
scipy/interpolate/_rgi.py ``_evaluate_linear``, scipy 1.15): per linear axis the interval index i
is the largest with grid[i] <= x (clamped to len-2) and y = (x - grid[i]) / (grid[i+1] - grid[i]);
the 2^5 hypercube corners are visited with the last axis fastest, (i, 1-y) before (i+1, y),
weight = ((((1 * w0) * w1) * w2) * w3) * w4 and value = value + table[corner] * weight.  Pinned
against the reference's own PowerInterpolator on a synthetic table (tests/golden/interp.npz; the
reference does not ship mergedGridSearchResultFinal.npy).
"""
from __future__ import annotations

import random as _random

import numpy as np

KEYS = ("Ua_ratio", "Cm_ratio", "Ca_ratio", "Hm_ratio", "air_temp", "mass_temp", "OD_temp",
        "HVAC_power", "hour", "date")
NEAREST = (0, 1, 2, 3, 7)
LINEAR = (4, 5, 6, 8, 9)


def synthetic_table(lens, seed: int = 2024) -> np.ndarray:
    """Deterministic stand-in for the Monte-Carlo table (W per house), C order over the axes."""
    rs = np.random.RandomState(seed)
    return 500.0 + 4000.0 * rs.random_sample(int(np.prod(lens)))


class OracleInterp:
    def __init__(self, grids, values, cfg_ua, cfg_cm, cfg_ca, cfg_hm):
        self.grids = [np.asarray(g, np.float64) for g in grids]
        lens = [len(g) for g in self.grids]
        self.values = np.asarray(values, np.float64).reshape(lens)
        self.cfg = (float(cfg_ua), float(cfg_cm), float(cfg_ca), float(cfg_hm))

    def clip(self, x):
        """clip_interpolation_point (interpolation.py:245-264), every axis."""
        out = []
        for v, g in zip(x, self.grids):
            hi, lo = np.max(g), np.min(g)
            out.append(hi if v > hi else (lo if v < lo else v))
        return out

    def point(self, x) -> float:
        """interpolate_grid_fast (interpolation.py:137-178) of one clipped point in KEYS order."""
        near = [int(np.argmin(np.abs(self.grids[a] - x[a]))) for a in NEAREST]
        idx, nd = [], []
        for a in LINEAR:
            g, v = self.grids[a], x[a]
            i = int(np.searchsorted(g, v, side="right")) - 1
            i = min(max(i, 0), len(g) - 2)
            idx.append(i)
            nd.append((v - g[i]) / (g[i + 1] - g[i]))
        sub = self.values[near[0], near[1], near[2], near[3], :, :, :, near[4], :, :]
        value = 0.0
        for c in range(32):
            w = 1.0
            e = []
            for k in range(5):
                b = (c >> (4 - k)) & 1
                w = w * (nd[k] if b else 1 - nd[k])
                e.append(idx[k] + b)
            value = value + sub[tuple(e)] * w
        return float(value)

    def house_point(self, ua, cm, ca, hm, T, Tm, target, od, cap, hour, date):
        """The clipped point interpolate_power builds for one house (interpolation.py:226-238)."""
        x = [ua / self.cfg[0], cm / self.cfg[1], ca / self.cfg[2], hm / self.cfg[3],
             T - target, Tm - target, od - target, cap, hour, date]
        return self.clip(x)


def point_time(t, solar_gain: bool):
    """(hour, date) of interpolate_power (interpolation.py:204-216)."""
    if not solar_gain:
        return 0.0, 0.0
    hour = (t - t.replace(hour=0, minute=0, second=0, microsecond=0)).total_seconds()
    return hour, float(t.timetuple().tm_yday)


def sample(n: int, k: int, rng=_random):
    """House ids and multi_factor (interpolation.py:218-224; draws k randoms when n > k)."""
    ids = list(range(n))
    if n <= k:
        return ids, 1.0
    return rng.choices(ids, k=k), float(n) / float(k)


def interpolate_power(interp: OracleInterp, pop: dict, T, Tm, od, t, solar_gain: bool, k: int,
                      rng=_random) -> float:
    """interpolate_power (interpolation.py:186-243) over an SoA population (keys Ua, Cm, Ca, Hm,
    target, cap)."""
    hour, date = point_time(t, solar_gain)
    ids, factor = sample(len(T), k, rng)
    base = 0.0
    for j in ids:
        x = interp.house_point(pop["Ua"][j], pop["Cm"][j], pop["Ca"][j], pop["Hm"][j], T[j], Tm[j],
                               pop["target"][j], od, pop["cap"][j], hour, date)
        base += interp.point(x)
    base *= factor
    return base


def load_files(bp):
    """The reference's three files (interp_parameters_dict.json, interp_dict_keys.csv, .npy)."""
    import csv
    import json

    with open(bp.path_parameter_dict) as f:
        params = json.load(f)
    with open(bp.path_dict_keys, newline="") as f:
        keys = next(csv.reader(f))
    grids = [params[k] for k in keys]
    values = np.load(bp.path_datafile, allow_pickle=False)
    return keys, grids, values
