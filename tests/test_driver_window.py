"""driver_window's vectorised series (Environment._driver_window_vec) == the per-tick driver loop,
bit for bit: tick drivers (t_od_prev, solar, s_prev, tick), and the env's datetime, OD temperature,
signal and RNG state afterwards.  Windows cross midnight and month ends; all three vectorisable
signal modes; solar gain on and off.  The GPU-marked copy runs the same check on the GPU box's
host CPU (NumPy's vectorised sin must equal its scalar sin there too)."""
import datetime as dt
import random

import numpy as np
import pytest

import golden_util as gu
from oracle_shard import OracleShard

CASES = [("sinusoidals", True, dt.datetime(2021, 1, 31, 23, 50), 600),
         ("sinusoidals", False, dt.datetime(2021, 6, 1, 7, 28, 30), 37),
         ("flat", True, dt.datetime(2021, 3, 14, 17, 59, 58), 200),
         ("regular_steps", True, dt.datetime(2021, 12, 31, 23, 59, 2), 333)]


def _env(mode, solar, start, seed):
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 10, "power_grid_prop.signal_properties.mode": mode,
                                     "cluster_prop.house_prop.solar_gain": solar})
    props.start_datetime = start
    props.start_datetime_mode = "fixed"
    return Environment(props, rng=random.Random(seed), _shard_factory=OracleShard)


def _check(mode, solar, start, n):
    a, b = _env(mode, solar, start, 11), _env(mode, solar, start, 11)
    assert a._vector_drivers_ok()
    for rep in range(2):
        wa = a._driver_window_vec(n)
        wb = b._driver_window_loop(n)
        np.testing.assert_array_equal(wa.a.view(np.uint64), wb.a.view(np.uint64))  # bitwise, incl. tick
        assert a.date_time == b.date_time
        assert float(a.current_od_temp) == float(b.current_od_temp)
        assert float(a.power_grid.current_signal) == float(b.power_grid.current_signal)
        assert a._solar == b._solar and a._tick == b._tick
        assert float(a._tod_prev) == float(b._tod_prev) and float(a._s_prev) == float(b._s_prev)
        assert a.rng.random() == b.rng.random()  # same number of draws


@pytest.mark.parametrize("mode,solar,start,n", CASES)
def test_vector_drivers_equal_loop(mode, solar, start, n):
    _check(mode, solar, start, n)


@pytest.mark.gpu
def test_vector_drivers_equal_loop_on_gpu_host():
    for case in CASES:
        _check(*case)
