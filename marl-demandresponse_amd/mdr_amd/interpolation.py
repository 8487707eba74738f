"""Interpolated base power: ``PowerInterpolator`` with the lookup on device.

Reference: server/app/core/environment/power_grid/interpolation.py:24-264 and the caller
PowerGrid.power_step (power_grid.py:60-66, 149-161).  Every ``interp_update_period`` seconds
(counting from ``period + 1`` at construction, so the reset's grid step interpolates) the base power
is re-estimated from ``interp_nb_agents`` houses drawn with ``random.choices`` (all houses, in order,
when the cluster is not larger), each house's power looked up in the Monte-Carlo table at its
(thermal ratios, air / mass / outdoor temperature offsets, cooling capacity, hour, day of year)
point, summed in sample order and scaled by N / k.

Files are the reference's own formats: ``path_parameter_dict`` (JSON, the axis values),
``path_dict_keys`` (CSV, the axis order), ``path_datafile`` (.npy, the table — 4,199,040 values on
the reference grid; the reference does not ship it, any table of the grid's shape loads).  The host
draws the ids and the per-tick scalars (they are the reference's RNG stream); the per-house clip /
nearest / multilinear lookup and the ordered sum run in ``k_interp_values`` / ``k_interp_sum``
(csrc/mdr_interp.hip) on the shard's device state.
"""
from __future__ import annotations

import csv
import json
import random as _random

import numpy as np

KEYS = ("Ua_ratio", "Cm_ratio", "Ca_ratio", "Hm_ratio", "air_temp", "mass_temp", "OD_temp",
        "HVAC_power", "hour", "date")
LINEAR = (4, 5, 6, 8, 9)


def load_tables(bp):
    """(axis value arrays in KEYS order, flat float64 table) from the three files."""
    with open(bp.path_parameter_dict) as f:
        params = json.load(f)
    with open(bp.path_dict_keys, newline="") as f:
        keys = next(csv.reader(f))
    if tuple(keys) != KEYS or tuple(params) != KEYS:
        # interpolate_grid_fast indexes the axes by position (interpolation.py:147-176)
        raise ValueError(f"interpolation axes must be {KEYS}, in this order, in both "
                         f"{bp.path_dict_keys} and {bp.path_parameter_dict}")
    grids = [np.asarray(params[k], np.float64) for k in keys]
    values = np.load(bp.path_datafile, allow_pickle=False)
    need = int(np.prod([len(g) for g in grids]))
    if values.size != need:
        raise ValueError(f"{bp.path_datafile}: {values.size} values, the grid needs {need}")
    for a in LINEAR:
        g = grids[a]
        if len(g) < 2 or np.any(np.diff(g) <= 0):
            raise ValueError(f"axis {KEYS[a]} must be strictly ascending with at least 2 points")
    return grids, np.ascontiguousarray(values, np.float64).reshape(-1)


def point_time(t, solar_gain: bool):
    """(hour, date) coordinates of interpolate_power (interpolation.py:204-216)."""
    if not solar_gain:  # "No solar gain - make it think it is midnight"
        return 0.0, 0.0
    hour = (t - t.replace(hour=0, minute=0, second=0, microsecond=0)).total_seconds()
    return hour, float(t.timetuple().tm_yday)


class Interpolator:
    """Host half of PowerInterpolator: the update clock, the sampling and the call into the device
    lookup (``evaluate(interp, ids, od, hour, date, factor) -> base power``)."""

    def __init__(self, base_power_props, house_prop, n_agents: int, rng=_random):
        self.bp = base_power_props
        self.hp = house_prop
        self.n = int(n_agents)
        self.rng = rng
        self.grids, self.values = load_tables(base_power_props)
        self.cfg = (house_prop.Ua, house_prop.Cm, house_prop.Ca, house_prop.Hm)
        self.since = base_power_props.interp_update_period + 1  # power_grid.py:64-66
        self.base = None

    def due(self, dt_seconds: int) -> bool:
        """Whether the next power_step interpolates (a pure look-ahead, draws nothing)."""
        return self.since + dt_seconds >= self.bp.interp_update_period

    def sample(self):
        """interpolation.py:218-224: all houses in order, or k draws of random.choices."""
        k = self.bp.interp_nb_agents
        if self.n <= k:
            return list(range(self.n)), 1.0
        return self.rng.choices(range(self.n), k=k), float(self.n) / float(k)

    def power_step(self, t, od: float, dt_seconds: int, evaluate) -> float:
        """PowerGrid.power_step (power_grid.py:149-161) in interpolation mode."""
        self.since += dt_seconds
        if self.since >= self.bp.interp_update_period:
            ids, factor = self.sample()
            hour, date = point_time(t, self.hp.solar_gain)
            self.base = float(evaluate(self, ids, od, hour, date, factor))
            self.since = 0
        return self.base
