"""Per-tick scalar drivers, computed on the host in the reference's own arithmetic and RNG order.

These are O(1) per tick (the same value for every house), so they stay on the host and reach the
kernels as ``mdr_tick`` arguments.  Each function keeps the reference's expression order so the
values are bit-identical (pinned by tests/test_oracle_golden.py and tests/test_host_logic.py):

  solar_gain      server/app/utils/utils.py:42-117
  od_temp         server/app/core/environment/environment.py:132-159
  Signal          server/app/core/environment/power_grid/signal_calculator.py:11-129
  GridSignal      server/app/core/environment/power_grid/power_grid.py:21-161 (interpolation
                  base power: mdr_amd/interpolation.py, lookup on device)
  deadband_l2     server/app/utils/utils.py:4-23 (scalar, for the reward normalisers)
"""
from __future__ import annotations

import datetime as _dt
import functools
import math as _math
import random as _random

import numpy as np

# CIBSE solar cooling load regression: (coefficient, x power, y power), summed in this order
SOLAR_TERMS = (
    (4.36579418e01, 0, 0), (1.58055357e02, 1, 0), (8.76635241e01, 0, 1), (-4.55944821e01, 2, 0),
    (3.24275366e00, 2, 1), (-4.56096472e-01, 2, 2), (-1.47795612e01, 0, 2), (4.68950855e00, 1, 2),
    (-3.73313090e01, 1, 1), (5.78827663e00, 3, 0), (1.04354810e00, 0, 3), (2.12969604e-02, 3, 1),
    (2.58881400e-03, 3, 2), (-5.11397219e-04, 3, 3), (1.56398008e-02, 2, 3),
    (-1.18302764e-01, 1, 3), (-2.71446436e-01, 4, 0), (-3.97855577e-02, 0, 4),
)


SOLAR_TERMS_ARRAY = np.array(SOLAR_TERMS, np.float64).reshape(-1)  # for the host-driver extension
SOLAR_TERMS_ARRAY.setflags(write=False)


def _powf(v: float, k: int) -> float:
    return v if k == 1 else v ** k


def solar_gain(t: _dt.datetime, window_area: float, shading_coeff: float) -> float:
    """Solar heat gain through the windows (W) at time t; identical for every house.

    It depends on (month, day, hour, minute) only, so a tick reuses the value of the previous
    ticks in the same minute (memoised: the same expression evaluated once, bit-identical)."""
    return _solar_memo(t.month, t.day, t.hour, t.minute, window_area, shading_coeff)


@functools.lru_cache(maxsize=1 << 16)
def _solar_memo(month: int, day: int, hour: int, minute: int, window_area: float, shading_coeff: float):
    x = hour + minute / 60 - 7.5
    if x < 0 or x > 10:
        load = 0
    else:
        y = month + day / 30 - 1
        load = SOLAR_TERMS[0][0]
        for c, i, j in SOLAR_TERMS[1:]:
            if i and j:
                load = load + _powf(x, i) * _powf(y, j) * c
            elif i:
                load = load + _powf(x, i) * c
            else:
                load = load + _powf(y, j) * c
    return window_area * shading_coeff * load


def od_temp(t: _dt.datetime, temp_prop, rng=_random):
    """Sinusoidal daily outdoor temperature + one gauss(0, temp_std) draw (consumes the RNG).
    The deterministic part depends on (hour, minute) only and is memoised."""
    temperature = _od_det(t.hour, t.minute, temp_prop.day_temp, temp_prop.night_temp, temp_prop.phase)
    temperature += rng.gauss(0, temp_prop.temp_std)
    return temperature


def solar_minute(month: int, day: int, hour: int, minute: int, window_area: float, shading_coeff: float):
    """solar_gain at a (month, day, hour, minute) (memoised)."""
    return _solar_memo(month, day, hour, minute, window_area, shading_coeff)


def od_day_list(temp_prop) -> list:
    """The daily outdoor-temperature curve (od_temp without the gauss draw) for every minute of the
    day, as a list of np.float64 (the scalar expression, evaluated once per process and config)."""
    return _od_day(temp_prop.day_temp, temp_prop.night_temp, temp_prop.phase)


@functools.lru_cache(maxsize=16)
def _od_day(day_temp, night_temp, phase):
    return [_od_det(m // 60, m % 60, day_temp, night_temp, phase) for m in range(1440)]


def od_day_array(temp_prop) -> np.ndarray:
    """od_day_list as a float64[1440] array (cached per config; the host-driver extension's table)."""
    return _od_day_a(temp_prop.day_temp, temp_prop.night_temp, temp_prop.phase)


@functools.lru_cache(maxsize=16)
def _od_day_a(day_temp, night_temp, phase):
    a = np.array(_od_day(day_temp, night_temp, phase), np.float64)
    a.setflags(write=False)
    return a


@functools.lru_cache(maxsize=64)
def solar_day_table(month: int, day: int, window_area: float, shading_coeff: float) -> np.ndarray:
    """Per-minute solar gain of one (month, day), filled on demand by the host-driver extension
    (NaN = not computed yet; each value is solar_minute's)."""
    return np.full(1440, np.nan, np.float64)


def od_day_floats(temp_prop) -> list:
    """od_day_list as Python floats (the same values: np.float64 -> float is exact; float
    arithmetic rounds like np.float64's and skips NumPy's scalar overhead)."""
    return _od_day_f(temp_prop.day_temp, temp_prop.night_temp, temp_prop.phase)


@functools.lru_cache(maxsize=16)
def _od_day_f(day_temp, night_temp, phase):
    return [float(x) for x in _od_day(day_temp, night_temp, phase)]


def _gauss_n_inline(rng, n: int, sigma: float) -> list:
    # random.Random.gauss (Lib/random.py, CPython 3.10) unrolled over n draws: the same pairs of
    # random() calls, the same cached second value (gauss_next), the same `mu + z * sigma` with
    # mu = 0 as the reference passes it (environment.py:132-159 via od_temp)
    random, log, sqrt, cos, sin = rng.random, _math.log, _math.sqrt, _math.cos, _math.sin
    out = []
    z = rng.gauss_next
    for _ in range(n):
        if z is None:
            x2pi = random() * _TWOPI
            g2rad = sqrt(-2.0 * log(1.0 - random()))
            out.append(0 + cos(x2pi) * g2rad * sigma)
            z = sin(x2pi) * g2rad
        else:
            out.append(0 + z * sigma)
            z = None
    rng.gauss_next = z
    return out


def _gauss_n_calls(rng, n: int, sigma: float) -> list:
    g = rng.gauss
    return [g(0, sigma) for _ in range(n)]


def _inline_matches() -> bool:
    """The unrolled draw is used only if it reproduces this interpreter's random.gauss exactly
    (values and the generator state after every draw)."""
    a, b = _random.Random(20240611), _random.Random(20240611)
    for n in (1, 2, 3, 7):
        if _gauss_n_inline(a, n, 1.7) != [b.gauss(0, 1.7) for _ in range(n)] or a.getstate() != b.getstate():
            return False
    return True


_TWOPI = 2.0 * _math.pi
_GAUSS_N = _gauss_n_inline if _inline_matches() else _gauss_n_calls


def gauss_n(rng, n: int, sigma: float) -> list:
    """[rng.gauss(0, sigma) for _ in range(n)], bit for bit and in the same RNG order (rng: a
    random.Random or the random module, whose bound functions share its hidden instance)."""
    inst = getattr(rng, "_inst", rng)  # the `random` module draws from random._inst
    if type(inst).gauss is not _random.Random.gauss:  # a subclass's own gauss: call it
        return _gauss_n_calls(inst, n, sigma)
    return _GAUSS_N(inst, n, sigma)


def od_daily(hour: int, minute: int, temp_prop):
    """The deterministic (daily sinusoid) part of od_temp, as np.float64."""
    return _od_det(hour, minute, temp_prop.day_temp, temp_prop.night_temp, temp_prop.phase)


@functools.lru_cache(maxsize=1 << 12)
def _od_det(hour: int, minute: int, day_temp, night_temp, phase):
    amplitude = (day_temp - night_temp) / 2.0
    bias = (day_temp + night_temp) / 2.0
    delay = -6.0 + phase
    time_day = hour + minute / 60.0
    return amplitude * np.sin(2 * np.pi * (time_day + delay) / 24.0) + bias


def deadband_l2(target, deadband, value):
    if target + deadband / 2 < value:
        return (value - (target + deadband / 2)) ** 2
    if target - deadband / 2 > value:
        return ((target - deadband / 2) - value) ** 2
    return 0.0


def reward_normalisers(reward_prop, house_prop):
    """(norm_temp, norm_sig) exactly as RewardsCalculator.compute_rewards computes them."""
    norm_t = deadband_l2(house_prop.target_temp, 0, house_prop.target_temp + 1)
    R = reward_prop.norm_reg_sig
    norm_s = deadband_l2(R, 0, 0.75 * R)
    return float(norm_t), float(norm_s)


def _seconds_of_day(t: _dt.datetime) -> int:
    return t.hour * 3600 + t.minute * 60 + t.second


@functools.lru_cache(maxsize=8)
def _day_stamps(year: int, month: int, day: int) -> np.ndarray:
    """time.mktime(t.timetuple()) % 86400 (signal_calculator.py:113) for every second t of the
    day, as the per-tick perlin path computes it: from midnight's stamp when the day has 86,400
    local seconds, else (a DST day) one mktime per second."""
    import time

    d0 = _dt.datetime(year, month, day)
    m0 = time.mktime(d0.timetuple())
    m1 = time.mktime((d0 + _dt.timedelta(days=1)).timetuple())
    sod = np.arange(86400, dtype=np.float64)
    if m1 - m0 == 86400.0:
        return (m0 + sod) % 86400
    return np.array([time.mktime((d0 + _dt.timedelta(seconds=k)).timetuple()) % 86400 for k in range(86400)])


class Signal:
    """Regulation-signal shape (signal_calculator.py), without the base-power part."""

    def __init__(self, signal_props, nb_agents: int, rng=_random):
        self.sp = signal_props
        self.nb_agents = nb_agents
        self.mode = signal_props.mode
        if self.mode == "perlin":
            from .perlin import Perlin

            # SignalCalculator draws the perlin seed from the global RNG (signal_calculator.py:24-31);
            # MDR_PERLIN_RESEED_GLOBAL=1: the pre-1.12 perlin_noise side effect on that generator
            import os

            side = os.environ.get("MDR_PERLIN_RESEED_GLOBAL", "0") == "1"
            self.perlin = Perlin(1, signal_props.nb_octaves, signal_props.octaves_step,
                                 signal_props.period, rng.random(), global_rng=rng if side else None)
        elif self.mode not in ("flat", "sinusoidals", "regular_steps"):
            raise ValueError(f"unknown signal mode {self.mode!r}")

    def __call__(self, base_power, t: _dt.datetime):
        sp = self.sp
        if self.mode == "flat":
            return base_power
        if self.mode == "sinusoidals":
            amplitudes = [base_power * r for r in sp.amplitude_ratios]
            if len(sp.periods) != len(amplitudes):
                raise ValueError("Power grid signal parameters: periods and amplitude_ratios lists "
                                 "should have the same length.")
            ts = _seconds_of_day(t)
            s = base_power
            for k, period in enumerate(sp.periods):
                s += amplitudes[k] * np.sin(2 * np.pi * ts / period)
            return s
        if self.mode == "regular_steps":
            amplitude = sp.amplitude_per_hvac * self.nb_agents
            ratio = base_power / amplitude
            return amplitude * np.heaviside((_seconds_of_day(t) % sp.period) - (1 - ratio) * sp.period, 1)
        # perlin: max(0, base * (1 + amplitude * noise(mktime(t) mod 86400)))
        import time

        stamp = time.mktime(t.timetuple()) % 86400
        return np.maximum(0, base_power + (base_power * sp.amplitude_ratios[0] * self.perlin.calculate_noise(stamp)))


class GridSignal:
    """PowerGrid (power_grid.py:21-161): base power x signal shape x artificial ratio, capped.

    ``grid_props`` is mutated like the reference's (its artificial_ratio compounds across resets,
    power_grid.py:44-49) because the reference does not copy it.
    """

    def __init__(self, grid_props, nb_agents: int, max_power: float, rng=_random, signal_fn=None,
                 house_prop=None):
        self.gp = grid_props
        self.nb_agents = nb_agents
        self.max_power = max_power
        grid_props.artificial_ratio = grid_props.artificial_ratio * \
            grid_props.artificial_signal_ratio_range ** (rng.random() * 2 - 1)
        self.current_signal = 0.0
        self._memo = {}
        self.signal = Signal(grid_props.signal_properties, nb_agents, rng)
        self.signal_fn = signal_fn
        bp = grid_props.base_power_props
        self.interp = None
        # evaluate(interp, ids, od, hour, date, factor) -> base power: the device lookup, set by the
        # Environment that owns the state (interpolation mode only)
        self.evaluate = None
        if bp.mode == "interpolation":
            from .interpolation import Interpolator

            if house_prop is None:
                raise ValueError("interpolation base power needs the house properties (ratio denominators)")
            self.interp = Interpolator(bp, house_prop, nb_agents, rng)  # power_grid.py:60-66
        elif bp.mode != "constant":
            raise ValueError(f"unknown base power mode {bp.mode!r}")

    def needs_state(self, dt_seconds: int) -> bool:
        """True if the next step interpolates, i.e. reads the post-step house state."""
        return self.interp is not None and self.interp.due(dt_seconds)

    def base_power(self, t=None, od=None, dt_seconds: int = 0):
        """PowerGrid.power_step (power_grid.py:130-161)."""
        if self.interp is not None:
            return self.interp.power_step(t, od, dt_seconds, self.evaluate)
        return self.gp.base_power_props.avg_power_per_hvac * self.nb_agents

    def step(self, t: _dt.datetime, od=None, dt_seconds: int = 0):
        base = self.base_power(t, od, dt_seconds)
        key = None
        if self.signal_fn is None and self.signal.mode != "perlin":
            # flat / sinusoidals / regular_steps depend on (base, seconds of day) only: memoised
            key = (base, _seconds_of_day(t) if self.signal.mode != "flat" else 0,
                   self.gp.artificial_ratio, self.max_power)
            hit = self._memo.get(key)
            if hit is not None:
                self.current_signal = hit
                return hit
        s = self.signal_fn(base, t) if self.signal_fn is not None else self.signal(base, t)
        s = s * self.gp.artificial_ratio
        self.current_signal = np.minimum(s, self.max_power)
        if key is not None:
            if len(self._memo) > (1 << 17):
                self._memo.clear()
            self._memo[key] = self.current_signal
        return self.current_signal

    def series_ok(self) -> bool:
        """The signal has a per-second-of-day table: constant base power, no caller signal_fn, and
        perlin only without the pre-1.12 global-RNG side effect (its draws interleave with the
        per-tick gauss draws)."""
        sig = self.signal
        return (self.interp is None and self.signal_fn is None and
                (sig.mode != "perlin" or sig.perlin.noise_list[0].global_rng is None))

    def day_table(self, date=None) -> np.ndarray:
        """current_signal after a step at every second of the day ``date`` (constant base power),
        cached per (base, artificial ratio, cap) — and per date in perlin mode, whose noise follows
        time.mktime (local time: a DST day has other stamps)."""
        dkey = (date.year, date.month, date.day) if self.signal.mode == "perlin" else None
        if dkey is None and date is None and self.signal.mode == "perlin":
            raise ValueError("a perlin day table needs its date")
        key = (self.base_power(), self.gp.artificial_ratio, self.max_power, dkey)
        if getattr(self, "_day_key", None) != key:
            sod = np.arange(86400, dtype=np.int64)
            stamps = _day_stamps(*dkey) if dkey is not None else None
            self._day_tab = self.signal_series(sod, stamps)
            self._day_key = key
        return self._day_tab

    def signal_series(self, sod, stamps=None) -> np.ndarray:
        """``step`` at a series of ticks (seconds of day ``sod``, int64 array; perlin: the ticks'
        time.mktime(t) % 86400 ``stamps``) for a constant base power: the same IEEE operations as
        the per-tick path, elementwise (float64 array)."""
        base = self.base_power()
        sp = self.signal.sp
        mode = self.signal.mode
        n = len(sod)
        if mode == "flat":
            s = np.full(n, base, np.float64)
        elif mode == "sinusoidals":
            amplitudes = [base * r for r in sp.amplitude_ratios]
            if len(sp.periods) != len(amplitudes):
                raise ValueError("Power grid signal parameters: periods and amplitude_ratios lists "
                                 "should have the same length.")
            s = np.full(n, base, np.float64)
            for k, period in enumerate(sp.periods):
                s = s + amplitudes[k] * np.sin(2 * np.pi * sod / period)
        elif mode == "regular_steps":
            amplitude = sp.amplitude_per_hvac * self.nb_agents
            ratio = base / amplitude
            s = amplitude * np.heaviside((sod % sp.period) - (1 - ratio) * sp.period, 1)
        elif mode == "perlin":
            noise = self.signal.perlin.calculate_noise_array(stamps)
            s = np.maximum(0, base + (base * sp.amplitude_ratios[0] * noise))
        else:
            raise ValueError(f"no series form for signal mode {mode!r}")
        s = s * self.gp.artificial_ratio
        return np.minimum(s, self.max_power)

    def get_obs(self):
        return {"reg_signal": self.current_signal}
