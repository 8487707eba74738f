"""CPU restatement of the reference environment step — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle (and the ``cpu_baseline`` "port" timed by ``bench.py``).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import it; the
product path (``mdr_amd``) never does, and fails loudly when its HIP library is missing.

It restates ``ALLabMTL/marl-demandresponse`` ``server/app`` (v2) vectorised over houses with NumPy
float64, keeping the reference's floating-point operation order so results agree to ~1e-13 (only
``exp`` may differ by an ulp; ``b**2`` is ``b*b`` here vs libm ``pow`` in the reference).

Pinned by the golden fixtures in ``tests/golden/`` that ``tests/golden/make_golden.py`` generated
by running the reference itself in the build container (see tests/test_oracle_golden.py).

Reference map (file:line relative to /root/reference):
  hvac_step            server/app/core/environment/cluster/hvac.py:43-64
  heat / power         server/app/core/environment/cluster/hvac.py:85-111
  update_temperature   server/app/core/environment/cluster/building.py:141-222
  solar_gain           server/app/utils/utils.py:42-117
  od_temp              server/app/core/environment/environment.py:132-159
  signal_*             server/app/core/environment/power_grid/signal_calculator.py:33-129
                       (perlin: oracle/perlin_np.py, the package's published algorithm — parity unpinned)
  grid_step            server/app/core/environment/power_grid/power_grid.py:80-161
  deadband_l2          server/app/utils/utils.py:4-23
  rewards              server/app/core/environment/rewards_calculator.py:29-203
  comm_links           server/app/core/environment/cluster/agent_communication_builder.py:36-203
  reset / noise        server/app/core/environment/environment.py:49-70,161-194;
                       server/app/core/environment/cluster/building.py:224-267; hvac.py:66-70
  norm_vector          server/app/utils/norm.py:31-218
  controllers          server/app/core/agents/controllers/bangbang_controllers.py:25-89;
                       server/app/core/agents/controllers/greedy_myopic_controller.py:67-104
"""
from __future__ import annotations

import datetime as _dt
import math
import random as _random
from typing import Dict, List, Optional

import numpy as np

# ------------------------------------------------------------------------------- HVAC FSM


def hvac_step(on, lock, sso, action, L: int, dt: int):
    """Lockout state machine, vectorised (hvac.py:43-64). Returns new (on, lock, sso)."""
    on = np.asarray(on, bool)
    action = np.asarray(action, bool)
    sso = np.asarray(sso, np.int64)
    sso = np.where(on, sso, sso + dt)
    locked = ~(on | (sso >= L))
    new_on = ~locked & action
    sso = np.where(new_on, 0, sso)
    new_lock = locked | (~locked & ~action & (sso + dt < L))
    return new_on, new_lock, sso


def heat_transfer(on, cap, lcf):
    """hvac.py:85-99: -1 * cap / (1 + lcf) when on, else 0."""
    q_on = (-1 * np.asarray(cap, np.float64)) / (1 + lcf)
    return np.where(on, q_on, 0.0)


def power(on, cap, cop):
    """hvac.py:101-111 + environment_properties.py:92-98 (cap / cop when on)."""
    return np.where(on, np.asarray(cap, np.float64) / cop, 0.0)


# ------------------------------------------------------------------------------- thermal


def update_temperature(T, Tm, Ua, Ca, Cm, Hm, q_hvac, G, Tod, dt):
    """2-node RC step (building.py:141-222), reference operation order, float64."""
    od_k = Tod + 273
    t_k = T + 273
    tm_k = Tm + 273
    Qa = q_hvac + G
    a = Cm * Ca / Hm
    b = Cm * (Ua + Hm) / Hm + Ca
    c = Ua
    d = Qa + Ua * od_k  # Qm (=0) + Qa + Ua*odK
    disc = np.sqrt(b * b - 4 * a * c)
    r1 = (-b + disc) / (2 * a)
    r2 = (-b - disc) / (2 * a)
    dTA0dt = Hm * tm_k / Ca - (Ua + Hm) * t_k / Ca + Ua * od_k / Ca + Qa / Ca
    A1 = (r2 * t_k - dTA0dt - r2 * d / c) / (r2 - r1)
    A2 = t_k - d / c - A1
    A3 = r1 * Ca / Hm + (Ua + Hm) / Hm
    A4 = r2 * Ca / Hm + (Ua + Hm) / Hm
    e1 = np.exp(r1 * dt)
    e2 = np.exp(r2 * dt)
    t_new = A1 * e1 + A2 * e2 + d / c
    tm_new = A1 * A3 * e1 + A2 * A4 * e2 + 0.0 + d / c
    return t_new - 273, tm_new - 273


# ------------------------------------------------------------------------------- scalar drivers

# (coefficient, power of x, power of y) in the reference's summation order (utils.py:63-105)
_SOLAR_TERMS = (
    (4.36579418e01, 0, 0), (1.58055357e02, 1, 0), (8.76635241e01, 0, 1), (-4.55944821e01, 2, 0),
    (3.24275366e00, 2, 1), (-4.56096472e-01, 2, 2), (-1.47795612e01, 0, 2), (4.68950855e00, 1, 2),
    (-3.73313090e01, 1, 1), (5.78827663e00, 3, 0), (1.04354810e00, 0, 3), (2.12969604e-02, 3, 1),
    (2.58881400e-03, 3, 2), (-5.11397219e-04, 3, 3), (1.56398008e-02, 2, 3),
    (-1.18302764e-01, 1, 3), (-2.71446436e-01, 4, 0), (-3.97855577e-02, 0, 4),
)


def _pw(v: float, k: int) -> float:
    return v if k == 1 else v ** k


def solar_gain(t: _dt.datetime, window_area: float, shading_coeff: float) -> float:
    x = t.hour + t.minute / 60 - 7.5
    if x < 0 or x > 10:
        load = 0
    else:
        y = t.month + t.day / 30 - 1
        load = None
        for c, i, j in _SOLAR_TERMS:
            if i and j:
                term = _pw(x, i) * _pw(y, j) * c
            elif i:
                term = _pw(x, i) * c
            elif j:
                term = _pw(y, j) * c
            else:
                term = c
            load = term if load is None else load + term
    return window_area * shading_coeff * load


def od_temp(t: _dt.datetime, tp, rng) -> float:
    amp = (tp.day_temp - tp.night_temp) / 2.0
    bias = (tp.day_temp + tp.night_temp) / 2.0
    delay = -6.0 + tp.phase
    hour = t.hour + t.minute / 60.0
    temp = amp * np.sin(2 * np.pi * (hour + delay) / 24.0) + bias
    return temp + rng.gauss(0, tp.temp_std)


def _tsec(t: _dt.datetime) -> int:
    return t.hour * 3600 + t.minute * 60 + t.second


def signal(mode: str, sp, base: float, t: _dt.datetime, nb_agents: int, perlin=None) -> float:
    if mode == "flat":
        return base
    if mode == "sinusoidals":
        if len(sp.periods) != len(sp.amplitude_ratios):
            raise ValueError("periods / amplitude_ratios length mismatch")
        amps = [base * r for r in sp.amplitude_ratios]
        ts = _tsec(t)
        s = base
        for k, period in enumerate(sp.periods):
            s += amps[k] * np.sin(2 * np.pi * ts / period)
        return s
    if mode == "regular_steps":
        amp = sp.amplitude_per_hvac * nb_agents
        ratio = base / amp
        per = sp.period
        return amp * np.heaviside((_tsec(t) % per) - (1 - ratio) * per, 1)
    if mode == "perlin" and perlin is not None:  # signal_calculator.py:100-115 (parity unpinned)
        import time

        stamp = time.mktime(t.timetuple()) % 86400
        return np.maximum(0, base + (base * sp.amplitude_ratios[0] * perlin.calculate_noise(stamp)))
    raise NotImplementedError(f"signal mode {mode!r} is not restated")


# ------------------------------------------------------------------------------- rewards


def deadband_l2(target, deadband, value):
    target = np.asarray(target, np.float64)
    value = np.asarray(value, np.float64)
    hi = target + deadband / 2
    lo = target - deadband / 2
    return np.where(hi < value, (value - hi) ** 2, np.where(lo > value, (lo - value) ** 2, 0.0))


def _deadband_l2_scalar(target, deadband, value):
    if target + deadband / 2 < value:
        return (value - (target + deadband / 2)) ** 2
    if target - deadband / 2 > value:
        return ((target - deadband / 2) - value) ** 2
    return 0.0


def temp_penalties(mode: str, pen, pp):
    """Per-house temperature penalty for each mode (rewards_calculator.py:46-133)."""
    n = pen.shape[0]
    if mode == "individual_L2":
        return pen
    common_l2 = 0.0
    for v in pen:  # sequential sum of pen/N (reference order)
        common_l2 += v / n
    common_max = 0.0
    for v in pen:
        if v > common_max:
            common_max = v
    if mode == "common_L2":
        return np.full(n, common_l2)
    if mode == "common_max_error":
        return np.full(n, common_max)
    if mode == "mixture":
        a, b, c = pp.alpha_ind_l2, pp.alpha_common_l2, pp.alpha_common_max
        return (a * pen + b * common_l2 + c * common_max) / (a + b + c)
    raise ValueError(mode)


def rewards(T, target, deadband, P, S_prev, rp, target_cfg):
    n = T.shape[0]
    pen = deadband_l2(target, deadband, T)
    tp = temp_penalties(rp.penalty_props.mode, pen, rp.penalty_props)
    sig_pen = ((P - S_prev) / n) ** 2
    norm_t = _deadband_l2_scalar(target_cfg, 0, target_cfg + 1)
    norm_s = _deadband_l2_scalar(rp.norm_reg_sig, 0, 0.75 * rp.norm_reg_sig)
    return -1 * (rp.alpha_temp * tp / norm_t + rp.alpha_sig * sig_pen / norm_s)


# ------------------------------------------------------------------------------- comm graph


def nb_comm(cp) -> int:
    return int(min(cp.agents_comm_prop.max_nb_agents_communication, cp.nb_agents - 1))


def comm_links(cp, rng) -> Optional[List[List[int]]]:
    """Neighbour table per house (agent_communication_builder.py). None for random_sample."""
    n = cp.nb_agents
    ac = cp.agents_comm_prop
    k = nb_comm(cp)
    mode = ac.mode
    if mode == "neighbours":
        lo, hi = k // 2, (k + 1) // 2
        return [[(i - lo + j) % n for j in range(lo)] + [(i + 1 + j) % n for j in range(hi)]
                for i in range(n)]
    if mode == "closed_groups":
        out = []
        for i in range(n):
            base = i - i % (k + 1)
            if base + k <= n:
                ids = [base + j for j in range(ac.max_nb_agents_communication + 1)]
            else:
                ids = [n - k - 1 + j for j in range(k + 1)]
            ids.remove(i)
            out.append(ids)
        return out
    if mode == "random_sample":
        return None
    if mode == "random_fixed":
        return [rng.sample([j for j in range(n) if j != i], k=k) for i in range(n)]
    if mode == "neighbours_2D":
        rs, dmax = ac.row_size, ac.max_communication_distance
        if n % rs != 0:
            raise ValueError("Neighbours 2D row_size must be a divisor of nb_agents")
        my = n // rs
        if dmax >= (rs + 1) // 2 or dmax >= (my + 1) // 2:
            raise ValueError("Neighbours 2D distance_comm too large")
        pat = [(dx, dy) for dx in range(-dmax, dmax + 1) for dy in range(-dmax, dmax + 1)
               if abs(dx) + abs(dy) <= dmax and (dx or dy)]
        return [[((i // rs + dy) % my) * rs + (i % rs + dx) % rs for dx, dy in pat] for i in range(n)]
    raise AttributeError(mode)


# ------------------------------------------------------------------------------- population


def draw_population(cp, rng):
    """Per-building noise in reference RNG order (building.py:224-267, hvac.py:66-70)."""
    hp = cp.house_prop
    nz = hp.noise_prop
    n = cp.nb_agents
    pop = {k: np.empty(n) for k in ("Ua", "Ca", "Cm", "Hm", "target", "cap", "init_air", "init_mass")}
    for i in range(n):
        pop["init_air"][i] = hp.init_air_temp + abs(rng.gauss(0, nz.std_start_temp))
        pop["init_mass"][i] = hp.init_mass_temp + abs(rng.gauss(0, nz.std_start_temp))
        pop["target"][i] = hp.target_temp + abs(rng.gauss(0, nz.std_target_temp))
        pop["Ua"][i] = rng.triangular(nz.factor_thermo_low, nz.factor_thermo_high, 1)
        pop["Cm"][i] = hp.Cm * rng.triangular(nz.factor_thermo_low, nz.factor_thermo_high, 1)
        pop["Ca"][i] = hp.Ca * rng.triangular(nz.factor_thermo_low, nz.factor_thermo_high, 1)
        pop["Hm"][i] = hp.Hm * rng.triangular(nz.factor_thermo_low, nz.factor_thermo_high, 1)
        pop["cap"][i] = rng.choices(hp.hvac_prop.noise_prop.cooling_capacity_list)[0]
    return pop


# ------------------------------------------------------------------------------- env


class OracleEnv:
    """Vectorised restatement of ``Environment`` (environment.py:23-194), SoA state."""

    def __init__(self, props, rng=None, population: Optional[dict] = None):
        """``population`` (keys Ua, Ca, Cm, Hm, target, cap) replaces the RNG draw of the
        per-building noise (used for synthetic bench populations); everything else is as the
        reference."""
        self.p = props
        self.rng = rng if rng is not None else _random
        self.n = props.cluster_prop.nb_agents
        self._pop0 = population
        self.reset()

    # environment.py:49-70
    def reset(self):
        p, cp, hp = self.p, self.p.cluster_prop, self.p.cluster_prop.house_prop
        n = self.n
        self.links = comm_links(cp, self.rng)
        self.max_power = 0.0
        self.P = 0.0
        pre = hp.hvac_prop.cooling_capacity / hp.hvac_prop.cop
        for _ in range(n):
            self.P += pre
            self.max_power += pre
        if self.links is None:  # Cluster.reset() -> get_obs() draws in random_sample mode
            self._random_links()
        self.date = p.start_datetime
        if p.start_datetime_mode == "random":
            days = self.rng.randrange(364)
            secs = self.rng.randrange(86400)
            self.date = p.start_datetime + _dt.timedelta(days=days, seconds=secs)
        self.pop = draw_population(cp, self.rng) if self._pop0 is None else \
            {k: np.array(v, np.float64) for k, v in self._pop0.items()}
        self.T = np.full(n, float(hp.init_air_temp))
        self.Tm = np.full(n, float(hp.init_mass_temp))
        self.on = np.ones(n, bool)
        self.lock = np.zeros(n, bool)
        self.sso = np.zeros(n, np.int64)
        self.G = 0.0
        self.Tod = od_temp(self.date, p.temp_prop, self.rng)
        gp = p.power_grid_prop
        gp.artificial_ratio = gp.artificial_ratio * gp.artificial_signal_ratio_range ** (
            self.rng.random() * 2 - 1)
        self._perlin = None
        sp = gp.signal_properties
        if sp.mode == "perlin":  # SignalCalculator draws its seed next (signal_calculator.py:24-31)
            from .perlin_np import PerlinSignal

            self._perlin = PerlinSignal(sp.nb_octaves, sp.octaves_step, sp.period, self.rng.random())
        self.S = 0.0
        self._interp_since = gp.base_power_props.interp_update_period + 1  # power_grid.py:64-66
        self._grid_step()
        self.cur_links = self._links_for_obs()
        return self.obs()

    def _random_links(self):
        k = nb_comm(self.p.cluster_prop)
        return [self.rng.sample([j for j in range(self.n) if j != i], k=k) for i in range(self.n)]

    def _links_for_obs(self):
        return self.links if self.links is not None else self._random_links()

    def _grid_step(self):
        """PowerGrid.step (power_grid.py:80-161); interpolation mode via oracle/interp_np.py."""
        gp = self.p.power_grid_prop
        bp = gp.base_power_props
        if bp.mode == "interpolation":
            from . import interp_np as IN

            if getattr(self, "_interp", None) is None:
                keys, grids, values = IN.load_files(bp)
                hp = self.p.cluster_prop.house_prop
                self._interp = IN.OracleInterp(grids, values, hp.Ua, hp.Cm, hp.Ca, hp.Hm)
            self._interp_since += self.p.time_step.seconds
            if self._interp_since >= bp.interp_update_period:
                self._base = IN.interpolate_power(self._interp, self.pop, self.T, self.Tm, self.Tod, self.date,
                                                  self.p.cluster_prop.house_prop.solar_gain,
                                                  bp.interp_nb_agents, self.rng)
                self._interp_since = 0
            base = self._base
        elif bp.mode != "constant":
            raise ValueError(f"unknown base power mode {bp.mode!r}")
        else:
            base = bp.avg_power_per_hvac * self.n
        s = signal(gp.signal_properties.mode, gp.signal_properties, base, self.date, self.n, self._perlin)
        s = s * gp.artificial_ratio
        self.S = np.minimum(s, self.max_power)

    # environment.py:72-108
    def step(self, actions):
        p, hp = self.p, self.p.cluster_prop.house_prop
        hv = hp.hvac_prop
        dts = p.time_step.seconds
        self.date = self.date + p.time_step
        self.on, self.lock, self.sso = hvac_step(self.on, self.lock, self.sso, actions,
                                                 hv.lockout_duration, dts)
        q = heat_transfer(self.on, self.pop["cap"], hv.latent_cooling_fraction)
        self.G = solar_gain(self.date, hp.window_area, hp.shading_coeff) if hp.solar_gain else 0.0
        self.T, self.Tm = update_temperature(self.T, self.Tm, self.pop["Ua"], self.pop["Ca"],
                                             self.pop["Cm"], self.pop["Hm"], q, self.G, self.Tod, dts)
        pw = power(self.on, self.pop["cap"], hv.cop)
        P = 0.0
        for v in pw:  # sequential, index order (cluster.py:82-88)
            P += v
        self.P = P
        if self.links is None:  # discarded Cluster.get_obs() in Cluster.step (cluster.py:89)
            self._random_links()
        self.Tod = od_temp(self.date, p.temp_prop, self.rng)
        rew = rewards(self.T, self.pop["target"], hp.deadband, self.P, self.S, p.reward_prop,
                      hp.target_temp)
        self._grid_step()
        self.cur_links = self._links_for_obs()
        return self.obs(), rew

    def obs(self) -> dict:
        return {"T": self.T.copy(), "Tm": self.Tm.copy(), "on": self.on.copy(),
                "lock": self.lock.copy(), "sso": self.sso.copy(), "P": float(self.P),
                "S": float(self.S), "Tod": float(self.Tod), "G": float(self.G), "date": self.date}

    def norm_vector(self) -> np.ndarray:
        return norm_vector(self.p, self.pop, self.obs(), self.cur_links)


# ------------------------------------------------------------------------------- obs vector


def norm_vector(p, pop, o, links) -> np.ndarray:
    """``norm_state_dict`` (norm.py:178-218) for all houses, float64 [N, F]."""
    n = p.cluster_prop.nb_agents
    has = links is not None and len(links) > 0 and len(links[0]) > 0
    return norm_vector_rows(p, pop, o, np.arange(n), links if has else None)


def norm_vector_rows(p, pop, o, rows, links_rows) -> np.ndarray:
    """``norm_state_dict`` (norm.py:178-218) of the houses ``rows`` only, float64 [len(rows), F];
    ``links_rows``: their neighbour ids [len(rows), k] (None: no messages).  State and population
    arrays cover the whole cluster (normalisers use the cluster size nb_agents)."""
    cp, hp = p.cluster_prop, p.cluster_prop.house_prop
    hv = hp.hvac_prop
    sp, mp = p.state_prop, cp.message_prop
    R = p.reward_prop.norm_reg_sig
    L = hv.lockout_duration
    n = cp.nb_agents
    rows = np.asarray(rows, np.int64)
    m = rows.shape[0]
    cols = [o["on"][rows].astype(np.float64), o["lock"][rows].astype(np.float64),
            np.trunc(o["sso"][rows] / L), np.full(m, float(int(L / L)))]
    if sp.hvac:
        cols += [np.full(m, hv.cop / hv.cop), np.full(m, hv.latent_cooling_fraction / hv.latent_cooling_fraction)]
    cols += [np.full(m, o["P"] / R), np.full(m, o["S"] / (R * n)), np.full(m, float(hp.deadband)),
             (o["T"][rows] - 20) / 5, (o["Tm"][rows] - 20) / 5, (pop["target"][rows] - 20) / 5]
    if sp.solar_gain:
        cols.append(np.full(m, o["G"] / 1000))
    if sp.thermal:
        cols += [pop["Ua"][rows] / hp.Ua, pop["Ca"][rows] / hp.Ca, pop["Cm"][rows] / hp.Cm, pop["Hm"][rows] / hp.Hm]
        cols.append(np.full(m, (o["Tod"] - 20) / 5))
    base = np.stack(cols, 1)
    if links_rows is None:
        return base
    idx = np.asarray(links_rows, np.int64)  # [m, k]
    curr = np.where(o["on"], pop["cap"] / hv.cop, 0.0)
    mx = pop["cap"] / hv.cop
    per = [(o["T"][idx] - pop["target"][idx]) / 5, np.trunc(o["sso"][idx] / L), curr[idx] / R, mx[idx] / R]
    if mp.thermal:
        per += [pop["Ua"][idx] / hp.Ua, pop["Ca"][idx] / hp.Ca, pop["Cm"][idx] / hp.Cm, pop["Hm"][idx] / hp.Hm]
    if mp.hvac:
        k = idx.shape[1]
        per += [np.full((m, k), hv.cop), np.full((m, k), hv.latent_cooling_fraction),
                np.full((m, k), float(hv.cooling_capacity))]
    msg = np.stack(per, 2).reshape(m, -1)
    return np.concatenate([base, msg], 1)


# ------------------------------------------------------------------------------- controllers


def bangbang(T, target):
    """BangBangController.act (bangbang_controllers.py:54-65)."""
    return np.asarray(T) > np.asarray(target)


def deadband_bangbang(T, target, deadband, on):
    """DeadbandBangBangController.act (bangbang_controllers.py:25-42)."""
    T = np.asarray(T)
    lo = np.asarray(target) - deadband / 2
    hi = np.asarray(target) + deadband / 2
    return np.where(T < lo, False, np.where(T > hi, True, np.asarray(on, bool)))


def greedy(T, target, cap, cop, lock, S):
    """GreedyMyopic.get_action (greedy_myopic_controller.py:67-104). Stable tie order."""
    key = -(np.asarray(T) - np.asarray(target))
    order = np.argsort(key, kind="stable")
    p = np.asarray(cap, np.float64) / cop
    act = np.zeros(len(key), bool)
    tot = 0
    for i in order:
        if p[i] + tot < S or abs(p[i] + tot - S) < abs(tot - S) and not lock[i]:
            tot += p[i]
            act[i] = True
    return act
