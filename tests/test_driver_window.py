"""driver_window's vectorised series (Environment._driver_window_vec) == the per-tick driver loop,
bit for bit: tick drivers (t_od_prev, solar, s_prev, tick), and the env's datetime, OD temperature,
signal and RNG state afterwards.  Windows cross midnight and month ends; all three vectorisable
signal modes and perlin (its restated noise tabulated per date, mdr_amd/perlin.py); solar gain on and
off.  The GPU-marked copy runs the same check on the GPU box's host CPU (NumPy's vectorised sin
must equal its scalar sin there too)."""
import datetime as dt
import random

import numpy as np
import pytest

import golden_util as gu
from oracle_shard import OracleShard

CASES = [("sinusoidals", True, dt.datetime(2021, 1, 31, 23, 50), 600),
         ("sinusoidals", False, dt.datetime(2021, 6, 1, 7, 28, 30), 37),
         ("flat", True, dt.datetime(2021, 3, 14, 17, 59, 58), 200),
         ("regular_steps", True, dt.datetime(2021, 12, 31, 23, 59, 2), 333),
         ("flat", True, dt.datetime(2021, 5, 9, 6, 0), 30000),  # 33 h: every daylight minute's solar gain
         ("perlin", True, dt.datetime(2021, 1, 31, 23, 50), 600),  # perlin day tables of two dates
         ("perlin", False, dt.datetime(2021, 8, 2, 11, 3, 30), 45)]


def _env(mode, solar, start, seed):
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 10, "power_grid_prop.signal_properties.mode": mode,
                                     "cluster_prop.house_prop.solar_gain": solar})
    props.start_datetime = start
    props.start_datetime_mode = "fixed"
    return Environment(props, rng=random.Random(seed), _shard_factory=OracleShard)


def _check(mode, solar, start, n, vec="_driver_window_vec"):
    a, b = _env(mode, solar, start, 11), _env(mode, solar, start, 11)
    assert a._vector_drivers_ok()
    for rep in range(2):
        wa = getattr(a, vec)(n)
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


@pytest.mark.parametrize("mode,solar,start,n", CASES)
def test_python_vector_drivers_equal_loop(mode, solar, start, n):
    _check(mode, solar, start, n, vec="_driver_window_vec_py")


def test_native_drivers_built():
    """The C host drivers (csrc/mdr_host.c) are the ones driver_window runs."""
    from mdr_amd import environment

    assert environment._host is not None


def test_native_drivers_module_rng_and_short_windows():
    """The `random` module as the generator (its hidden instance), a cached gauss_next carried
    across calls, windows of 1 and 2 ticks."""
    import random as R

    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 10, "power_grid_prop.signal_properties.mode": "sinusoidals"})
    props.start_datetime = dt.datetime(2021, 7, 4, 23, 59, 50)
    props.start_datetime_mode = "fixed"
    R.seed(5)
    a = Environment(props, rng=R, _shard_factory=OracleShard)
    R.seed(5)
    b = Environment(props, rng=R, _shard_factory=OracleShard)
    R.seed(7)
    R.gauss(0, 1)  # leaves a cached deviate
    st = R.getstate()
    outs = []
    for env, f in ((a, "_driver_window_vec"), (b, "_driver_window_loop")):
        R.setstate(st)
        rows = [getattr(env, f)(k).a.copy() for k in (2, 1, 3, 7)]
        outs.append((np.concatenate(rows).view(np.uint64), R.getstate()))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]


@pytest.mark.gpu
def test_vector_drivers_equal_loop_on_gpu_host():
    for case in CASES:
        _check(*case)


def test_overridden_gauss_uses_it():
    """A random.Random subclass with its own gauss: driver_window draws through that gauss (the C
    drivers and the unrolled draw restate CPython's gauss, so they are not used), equal to the
    per-tick loop."""
    from mdr_amd import environment

    class MyRandom(random.Random):
        def gauss(self, mu=0.0, sigma=1.0):
            return mu + sigma * (self.random() - 0.5)

    assert not environment._host_gauss_ok(MyRandom(3)) and environment._host_gauss_ok(random.Random(3))
    a, b = _env("sinusoidals", True, dt.datetime(2021, 4, 1, 12, 0), 11), _env("sinusoidals", True,
                                                                                dt.datetime(2021, 4, 1, 12, 0), 11)
    a.rng, b.rng = MyRandom(9), MyRandom(9)
    wa, wb = a.driver_window(50), b._driver_window_loop(50)
    np.testing.assert_array_equal(wa.a.view(np.uint64), wb.a.view(np.uint64))
    assert a.rng.random() == b.rng.random()
