"""Drop-in ``Environment`` on MI355X: the reference's reset/step object surface, HIP underneath.

Reference: server/app/core/environment/environment.py:23-194 (and the collaborators it calls,
cited per method).  Same constructor argument (an ``EnvironmentProperties``: ours from
``mdr_amd.config`` or the reference's own pydantic object), same ``reset() -> Dict[int, obs]``
and ``step(Dict[int, bool]) -> (Dict[int, obs], Dict[int, float])``, same attributes the server
reads (``init_props``, ``date_time``, ``current_od_temp``, ``cluster.current_power_consumption``,
``cluster.max_power``, ``cluster.buildings``, ``power_grid.current_signal``), same global-``random``
call order, so a seeded caller gets the reference's trajectory (tests/test_env_parity_gpu.py).

Fast paths (no per-house Python): ``step_tensor`` (device actions -> device rewards),
``obs_tensor`` (the ``norm_state_dict`` vector, float32 [N, F] on device) and ``rollout``
(many ticks per call, hipGraph-captured).
"""
from __future__ import annotations

import copy
import datetime as _dt
import random as _random
from collections.abc import Sequence
from types import SimpleNamespace
from typing import Dict, Optional

import numpy as np

from . import _lib as L
from . import config as cfgmod
from . import drivers
from . import population as popmod
from .drivers import GridSignal, od_temp, reward_normalisers, solar_gain
from .lazydict import LazyDict
from .shard import HipShard, encode_hvac

try:  # the rollout host drivers in C (csrc/mdr_host.c, built by build_ext.py); host code only
    from . import _mdr_host as _host
except ImportError:  # pragma: no cover - the Python loop computes the same values
    _host = None
if _host is not None:
    L.check_host_ext(_host)  # (a stale build is refused, as libmdr_hip.so is)
_HOST_ROLLOUT_NOT_CALLED = 1  # rollout1's rc_rollout when it did not call mdr_rollout (mdr_host.c)

ACTION_MODES = {"buffer": L.ACT_BUFFER, "random": L.ACT_RANDOM, "always_on": L.ACT_ALWAYS_ON,
                "bangbang": L.ACT_BANGBANG, "deadband_bangbang": L.ACT_DEADBAND_BANGBANG}


def _runs(key: np.ndarray):
    """(values of the runs of equal consecutive keys as ints, run index of every element)."""
    chg = np.empty(key.shape[0], bool)
    chg[0] = True
    np.not_equal(key[1:], key[:-1], out=chg[1:])
    return key[chg].tolist(), np.cumsum(chg) - 1



class _BuildingList(Sequence):
    """The parts of ``Building`` / ``HVAC`` the server reads (cluster.py:48-62), per house on access,
    from one host copy of the state taken when the list is created."""

    def __init__(self, env):
        self._env = env
        self._st = env._shard.host_state()
        self._prm = env._params_host()

    def __len__(self) -> int:
        return self._env._n_local

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        i = int(i)
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        st, prm, env = self._st, self._prm, self._env
        hp = env.init_props.cluster_prop.house_prop
        cap = env._cap_values[int(prm["cap_idx"][i])]
        hv = SimpleNamespace(turned_on=bool(st["on"][i]), lockout=bool(st["lock"][i]),
                             seconds_since_off=int(st["sso"][i]),
                             init_props=SimpleNamespace(cooling_capacity=cap, cop=hp.hvac_prop.cop,
                                                        max_consumption=cap / hp.hvac_prop.cop,
                                                        lockout_duration=hp.hvac_prop.lockout_duration))
        ip = SimpleNamespace(Ua=float(prm["ua"][i]), Ca=float(prm["ca"][i]), Cm=float(prm["cm"][i]),
                             Hm=float(prm["hm"][i]), target_temp=float(prm["target"][i]), deadband=hp.deadband)
        return SimpleNamespace(indoor_temp=float(st["T"][i]), current_mass_temp=float(st["Tm"][i]),
                               current_solar_gain=env._solar, init_props=ip, hvac=hv)


class TickWindow:
    """The per-tick drivers of a rollout window: one C-contiguous float64 [n, 4] array in the
    mdr_tick layout (t_od_prev, solar, s_prev as f64; tick as u64 bits), so the C ABI reads it in
    place — no per-tick Python objects."""

    __slots__ = ("a",)

    def __init__(self, a: np.ndarray):
        assert a.dtype == np.float64 and a.ndim == 2 and a.shape[1] == 4 and a.flags.c_contiguous
        self.a = a

    def __len__(self) -> int:
        return self.a.shape[0]

    @property
    def t_od_prev(self) -> np.ndarray:
        return self.a[:, 0]

    @property
    def solar(self) -> np.ndarray:
        return self.a[:, 1]

    @property
    def s_prev(self) -> np.ndarray:
        return self.a[:, 2]

    @property
    def tick(self) -> np.ndarray:
        return self.a[:, 3].view(np.uint64)

    def ptr(self) -> int:
        """Host address of the mdr_tick[n] array (valid while this object lives)."""
        return self.a.ctypes.data

    def struct(self, i: int) -> L.mdr_tick:
        r = self.a[i]
        return L.mdr_tick(float(r[0]), float(r[1]), float(r[2]), int(self.tick[i]))

    def __getitem__(self, sl: slice) -> "TickWindow":
        if not isinstance(sl, slice):
            raise TypeError("TickWindow slices only (use .struct(i) for one tick)")
        return TickWindow(np.ascontiguousarray(self.a[sl]))


def _host_gauss_ok(rng) -> bool:
    """The C host drivers restate CPython's random.gauss (its gauss_next cache, the generator's own
    random()); use them only when that is what the generator draws with: the ``random`` module or a
    random.Random whose gauss is not overridden, while the unrolled restatement is in use
    (drivers._GAUSS_N: chosen at import only if it reproduces this interpreter's gauss)."""
    inst = getattr(rng, "_inst", rng)
    return type(inst).gauss is _random.Random.gauss and drivers._GAUSS_N is drivers._gauss_n_inline


def shard_range(n: int, rank: int, world: int):
    """Contiguous house range of a rank: [r*n//w, (r+1)*n//w)."""
    lo = rank * n // world
    hi = (rank + 1) * n // world
    return lo, hi - lo


class _ClusterView:
    """The parts of ``Cluster`` (cluster.py:17-126) the server and controllers read."""

    def __init__(self, env: "Environment"):
        self._env = env

    @property
    def init_props(self):
        return self._env.init_props.cluster_prop

    @property
    def max_power(self) -> float:
        return self._env._max_power

    @property
    def current_power_consumption(self) -> float:
        return self._env._cluster_power()

    @property
    def buildings(self):
        return self._env._building_views()

    @property
    def agent_communicators(self):
        links = self._env._obs_links
        return {self._env._offset + i: [int(j) for j in row] for i, row in enumerate(links)} if links is not None else {}


class Environment:
    """Vectorised environment for N houses (one shard of them per process on multi-GPU)."""

    def __init__(self, env_props, device=None, rng=None, population: str = "reference",
                 seed: int = 0, signal_fn=None, rank: int = 0, world: int = 1, comm=None,
                 _shard_factory=None):
        self.init_props = copy.deepcopy(env_props)
        cfgmod.validate(self.init_props)
        if population not in ("reference", "synthetic"):
            raise ValueError("population must be 'reference' (host RNG, reference stream) or 'synthetic'")
        self.rng = rng if rng is not None else _random
        self._population = population
        self._seed = int(seed)
        self._signal_fn = signal_fn
        self.rank, self.world = int(rank), int(world)
        if world > 1 and comm is None:
            raise ValueError("a multi-shard Environment needs a comm (mdr_amd.distributed)")
        self._comm = comm
        self._gq_shard_fallbacks = 0  # sharded histogram-select calls decided by the all-gather form
        self._gq_force_sharded = False  # tests: the sharded greedy stages at world 1 (RCCL to self)
        self._device = device
        self._shard_factory = _shard_factory
        self._shard: Optional[HipShard] = None
        self.cluster = _ClusterView(self)
        self.reset(return_obs=False)  # the reference's __init__ resets and discards the obs

    # ------------------------------------------------------------------ geometry
    @property
    def n(self) -> int:
        return self.init_props.cluster_prop.nb_agents

    @property
    def n_local(self) -> int:
        return self._n_local

    @property
    def shard(self) -> HipShard:
        return self._shard

    # ------------------------------------------------------------------ reset
    def reset(self, return_obs: bool = True):
        """environment.py:49-70 (RNG order: SURVEY Appendix B).  ``return_obs=False`` skips the
        host-side dict materialisation (it draws nothing from the RNG) for tensor-API callers."""
        p = self.init_props
        cp, hp = p.cluster_prop, p.cluster_prop.house_prop
        hv = hp.hvac_prop
        rng = self.rng
        n = cp.nb_agents
        self._offset, self._n_local = shard_range(n, self.rank, self.world)
        # Cluster.reset (cluster.py:49-69): pre-noise power / max power, comm graph, get_obs()
        pre = hv.cooling_capacity / hv.cop
        seq = float(np.cumsum(np.full(n, pre, np.float64))[-1])  # sequential float sum
        self._max_power = seq
        self._P_host = seq
        self._P_dev_valid = False
        self._links = popmod.comm_links(cp, rng)
        if self._links is None:
            popmod.random_links(cp, rng)  # Cluster.reset() -> get_obs() draws in random_sample mode
        # Environment.apply_noise: randomize_date then per-building noise
        self.date_time = p.start_datetime
        if p.start_datetime_mode == "random":
            days = rng.randrange(364)
            secs = rng.randrange(86400)
            self.date_time = p.start_datetime + _dt.timedelta(days=days, seconds=secs)
        lo, nl = self._offset, self._n_local
        if self._population == "reference":
            pop = popmod.draw_reference(cp, rng)
            table, idx = popmod.cap_table(hv, pop["cap"][lo:lo + nl])
            local = {k: pop[k][lo:lo + nl] for k in ("ua", "ca", "cm", "hm", "target")}
        else:
            table, idx = popmod.cap_table(hv, ())
            local = None
        self._cap_values = table
        # outdoor temperature, grid, rewards calculator (environment.py:59-66)
        self.current_od_temp = od_temp(self.date_time, p.temp_prop, rng)
        self.power_grid = GridSignal(p.power_grid_prop, n, self._max_power, rng, self._signal_fn, hp)
        self.power_grid.evaluate = self._interp_evaluate
        self._norm_temp, self._norm_sig = reward_normalisers(p.reward_prop, hp)
        # device state (Building.reset / HVAC.reset: init temps, on, no lockout, sso = 0); before the
        # first grid step, which reads it in interpolation mode
        self._ensure_shard(table)
        sh = self._shard
        if local is not None:
            sh.upload(local, idx, np.full(nl, float(hp.init_air_temp)), np.full(nl, float(hp.init_mass_temp)),
                      encode_hvac(np.ones(nl, bool), np.zeros(nl, bool), np.zeros(nl, np.int64)))
        else:
            sh.populate(hp, table)
        self._host_params = None
        self._solar = 0.0
        self._tick = 0
        self._counts_ready = 0
        self._grid_pending = False
        self.power_grid.step(self.date_time, self.current_od_temp, p.time_step.seconds)  # first signal (:67-69)
        if self._vector_drivers_ok():  # rollout driver tables, built here rather than inside a rollout
            self.power_grid.day_table(self.date_time)
            drivers.od_day_list(p.temp_prop)
        self._obs_links = self._links if self._links is not None else popmod.random_links(cp, rng)
        return self.get_obs() if return_obs else None

    def _ensure_shard(self, cap_values):
        key = (tuple(cap_values), self._n_local)
        if self._shard is not None and self._shard_key == key:
            return
        if self._shard is not None:
            self._shard.close()
        factory = self._shard_factory or HipShard
        dev = self._device
        if dev is None:
            import torch

            dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cuda"
        self._shard = factory(self.init_props, self._n_local, self._offset, self.n, dev, cap_values,
                              seed=self._seed)
        self._shard_key = key
        if self._comm is not None and hasattr(self._comm, "attach"):
            self._comm.attach(self._shard)

    # ------------------------------------------------------------------ step
    def _tick_args(self) -> L.mdr_tick:
        return L.mdr_tick(float(self._tod_prev), float(self._solar), float(self._s_prev), self._tick)

    def step_tensor(self, actions=None, action_mode: str = "buffer", lookahead: Optional[str] = None,
                    ctrl: Optional[str] = None, ctrl_out=None, rewards=None):
        """One tick on device.  ``actions``: uint8/bool tensor [n_local] on the shard's device
        (``action_mode='buffer'``) or None with an in-kernel source ('random', 'always_on',
        'bangbang', 'deadband_bangbang').  Returns the device reward tensor (float64 [n_local]):
        ``rewards`` if given (a contiguous float64 [n_local] device tensor), else the shard's
        reward buffer (overwritten by the next tick).

        ``lookahead`` names the NEXT tick's in-kernel action source: its cluster-power counts
        are computed by this launch, so the next tick is a single kernel.  ``ctrl``: a controller
        evaluated on the post-step state ('bangbang' / 'deadband_bangbang' into ``ctrl_out``), or
        'greedy_keys': the next ``greedy_actions`` call's keys, prepared by this launch.
        """
        p = self.init_props
        hp = p.cluster_prop.house_prop
        sh = self._shard
        mode = ACTION_MODES[action_mode]
        if mode == L.ACT_BUFFER:
            if actions is None:
                raise ValueError("action_mode='buffer' needs an actions tensor")
            if actions.dtype != sh.action.dtype:
                actions = actions.to(sh.action.dtype)
            if actions.numel() != self._n_local:
                raise ValueError(f"actions must have {self._n_local} elements")
            actions = actions.contiguous()
        # environment.py:86-91: time advances, the cluster steps with the previous OD temp
        self.date_time = self.date_time + p.time_step
        self._solar = solar_gain(self.date_time, hp.window_area, hp.shading_coeff) if hp.solar_gain else 0.0
        self._tod_prev = self.current_od_temp
        self._s_prev = self.power_grid.current_signal
        tick = self._tick_args()
        if mode == L.ACT_BUFFER and self._counts_ready in (("actor", actions.data_ptr()), ("greedy", actions.data_ptr())):
            pass  # the actor / greedy launches that wrote these actions also counted their cluster power
        elif mode == L.ACT_BUFFER or self._counts_ready != mode:
            # phase 1 (unless the previous launch already counted this tick under the same source)
            if mode in (L.ACT_BUFFER, L.ACT_RANDOM, L.ACT_ALWAYS_ON):
                sh.power_counts(actions, mode, self._tick)
            else:
                self._bangbang_counts(mode)
        if self._comm is not None:
            self._comm.allreduce_counts(sh)
        la = ACTION_MODES[lookahead] if lookahead else 0
        cm = {None: 0, "bangbang": L.CTRL_BANGBANG, "deadband_bangbang": L.CTRL_DEADBAND_BANGBANG,
              "greedy_keys": L.CTRL_GREEDY_KEYS}[ctrl]
        if cm == L.CTRL_GREEDY_KEYS and self.world > 1:
            cm = 0  # (the sharded greedy gathers its rows itself)
        if rewards is not None and (rewards.dtype != sh.reward.dtype or rewards.numel() != self._n_local
                                    or not rewards.is_contiguous()):
            raise ValueError(f"rewards must be a contiguous float64 tensor of {self._n_local} elements")
        reward = sh.step(actions, mode, tick, lookahead=la, ctrl=cm, ctrl_out=ctrl_out, reward=rewards)
        if sh.penalty_mode != 0:
            sh.penalty_partials()
            if self._comm is not None:
                self._comm.allreduce_penalty(sh)
            sh.reward_finalize(tick, reward=reward)
        self._counts_ready = la
        self._P_dev_valid = True
        cp = p.cluster_prop
        if self._links is None:
            popmod.random_links(cp, self.rng)  # the discarded Cluster.get_obs() (cluster.py:89)
        self.current_od_temp = od_temp(self.date_time, p.temp_prop, self.rng)
        self.power_grid.step(self.date_time, self.current_od_temp, p.time_step.seconds)
        self._obs_links = self._links if self._links is not None else popmod.random_links(cp, self.rng)
        self._tick += 1
        return reward

    def _bangbang_counts(self, mode):
        # phase 1 for a bang-bang source: evaluate the controller on the current state on device
        import torch

        sh = self._shard
        T, tgt = sh.t_air, sh.target
        if mode == L.ACT_BANGBANG:
            a = T > tgt
        else:
            db = self.init_props.cluster_prop.house_prop.deadband
            on = (sh.hvac < 0)  # bit 31
            a = torch.where(T < tgt - db / 2, torch.zeros_like(on), torch.where(T > tgt + db / 2, torch.ones_like(on), on))
        sh.action.copy_(a.to(torch.uint8))
        sh.power_counts(sh.action, L.ACT_BUFFER, self._tick)

    def step(self, action_dict):
        """environment.py:72-108 — dict in, (obs dict, rewards dict) out."""
        import torch

        a = np.zeros(self._n_local, np.uint8)
        lo, nl = self._offset, self._n_local
        if isinstance(action_dict, dict):
            for k, v in action_dict.items():
                try:
                    j = int(k) - lo
                except (TypeError, ValueError):
                    continue
                if 0 <= j < nl and v:
                    a[j] = 1
        else:
            a[:] = np.asarray(action_dict, bool)[lo:lo + nl] if len(action_dict) == self.n else np.asarray(action_dict, bool)
        sh = self._shard
        sh.action.copy_(torch.from_numpy(a).to(sh.device))
        reward = self.step_tensor(sh.action)
        r = reward.cpu().numpy()
        rewards = LazyDict(lambda g: float(r[g - lo]), range(lo, lo + nl))
        return self.get_obs(), rewards

    # ------------------------------------------------------------------ many ticks per call
    def driver_window(self, n_ticks: int) -> "TickWindow":
        """Advance the host drivers up to n_ticks ahead (same RNG order as n calls of step) and
        return the per-tick drivers of a rollout as a ``TickWindow`` (the mdr_tick array the C
        ABI reads).  Valid when nothing else draws from the RNG between ticks (random_sample comm
        mode draws, so it is excluded).

        In interpolation base-power mode the window stops after a tick whose grid step reads the
        post-step house state: run the returned ticks on the device, then ``finish_grid_step()``."""
        if self._links is None:
            raise NotImplementedError("random_sample comm mode draws per tick; use step()")
        if self._grid_pending:
            raise RuntimeError("a deferred grid step is pending: run the previous window, then finish_grid_step()")
        if n_ticks >= 2 and self._vector_drivers_ok():
            return self._driver_window_vec(n_ticks)
        return self._driver_window_loop(n_ticks)

    def _vector_drivers_ok(self) -> bool:
        st = self.init_props.time_step
        return self.power_grid.series_ok() and st.microseconds == 0 and st.days == 0 and 0 < st.seconds < 86400

    def _driver_window_vec(self, n: int, launch=None):
        """driver_window for a constant base power and a flat / sinusoidal / regular-steps signal:
        the host-driver extension (csrc/mdr_host.c) when it is built, else the Python loop below
        (the same values bit for bit: tests/test_driver_window.py).  ``launch`` (Environment.rollout's
        direct sequence): the first day's ticks go through ``_host.rollout1``, which issues
        mdr_rollout_begin, computes them and — when the window ends that day — launches
        mdr_rollout itself; returns (TickWindow, launched) then."""
        if _host is None or not _host_gauss_ok(self.rng):
            return self._driver_window_vec_py(n)
        p = self.init_props
        hp = p.cluster_prop.house_prop
        tp, grid = p.temp_prop, self.power_grid
        od_tab = drivers.od_day_array(tp)
        dts = p.time_step.seconds
        d0 = self.date_time
        s = d0.hour * 3600 + d0.minute * 60 + d0.second
        rng = getattr(self.rng, "_inst", self.rng)  # the `random` module draws from random._inst
        solar_on, wa, shc = hp.solar_gain, hp.window_area, hp.shading_coeff
        buf = np.empty((n, 4), np.float64)
        tod, sig, sol = float(self.current_od_temp), float(grid.current_signal), 0.0
        tick0, done, day_off = self._tick, 0, 0
        while True:
            dd = d0 + _dt.timedelta(days=day_off) if day_off else d0
            sig_tab = grid.day_table(dd)  # (the tick's new datetime: its signal)
            sol_tab = drivers.solar_day_table(dd.month, dd.day, wa, shc) if solar_on else None
            if launch is not None and done == 0:
                rc_b, rc_r, k, s, tod, sig, sol = _host.rollout1(
                    *launch, rng, rng.random, tp.temp_std, n, s, dts, od_tab, sig_tab, sol_tab, dd.month, dd.day,
                    wa, shc, drivers.SOLAR_TERMS_ARRAY, tod, sig, sol, tick0, buf)
                L.check(rc_b, "mdr_rollout_begin")
                # rc_r: mdr_rollout's status (0 or a negative MDR_E*), or 1 = not called (the
                # window crossed midnight: the caller launches once the next day's drivers exist)
                if rc_r != _HOST_ROLLOUT_NOT_CALLED:
                    L.check(rc_r, "mdr_rollout")
                launched = rc_r == 0
            else:
                k, s, tod, sig, sol = _host.drivers(rng, rng.random, tp.temp_std, n - done, s, dts, od_tab, sig_tab,
                                                    sol_tab, dd.month, dd.day, wa, shc, drivers.SOLAR_TERMS_ARRAY,
                                                    tod, sig, sol, tick0 + done, buf[done:])
            done += k
            if done == n:
                break
            s -= 86400  # the next tick is on the next day
            day_off += 1
        self.date_time = d0 + p.time_step * n
        self._solar, self._tick = sol, tick0 + n
        self._tod_prev, self._s_prev = buf[n - 1, 0], buf[n - 1, 2]
        self.current_od_temp = np.float64(tod)
        grid.current_signal = np.float64(sig)
        return TickWindow(buf) if launch is None else (TickWindow(buf), launched)

    def _driver_window_vec_py(self, n: int) -> "TickWindow":
        """driver_window for a constant base power and a flat / sinusoidal / regular-steps signal:
        the same values as the per-tick loop, bit for bit (tests/test_driver_window.py), from
        per-day lookup tables built at reset — the regulation signal by second of the day
        (GridSignal.day_table) and the outdoor-temperature daily curve by minute
        (drivers.od_day_list) — plus the solar gain once per minute (memoised scalar code) and the
        n gauss draws in the reference order (nothing else draws in between).  A short Python
        loop: no per-tick objects beyond the draws, and no NumPy call per tick."""
        p = self.init_props
        hp = p.cluster_prop.house_prop
        tp, grid = p.temp_prop, self.power_grid
        sig_tab = grid.day_table(self.date_time)
        od_tab = drivers.od_day_floats(tp)
        gs = drivers.gauss_n(self.rng, n, tp.temp_std)  # the n draws, in order (nothing else draws)
        dts = p.time_step.seconds
        d0 = self.date_time
        s = d0.hour * 3600 + d0.minute * 60 + d0.second
        solar_on, wa, shc = hp.solar_gain, hp.window_area, hp.shading_coeff
        month, mday, day_off = d0.month, d0.day, 0
        sol, last_m = 0.0, -1
        # flat [t_od_prev, solar, s_prev, 0.0] * n, then one array; the tick column is set below
        tod, sig = float(self.current_od_temp), grid.current_signal
        flat = []
        push = flat.extend
        for g in gs:
            # environment.py:86-106: the new datetime's solar gain, the previous OD temperature
            # for the step, then one gauss for the new OD temperature and the new signal
            s += dts
            if s >= 86400:
                s -= 86400
                day_off += 1
                dd = d0 + _dt.timedelta(days=day_off)
                month, mday, last_m = dd.month, dd.day, -1
                sig_tab = grid.day_table(dd)
            m = s // 60
            if solar_on and m != last_m:
                sol = drivers.solar_minute(month, mday, m // 60, m % 60, wa, shc)
                last_m = m
            push((tod, sol, sig, 0.0))
            tod = od_tab[m] + g
            sig = sig_tab[s]
        buf = np.array(flat, np.float64).reshape(n, 4)
        tick0 = self._tick
        buf[:, 3].view(np.uint64)[:] = np.arange(tick0, tick0 + n, dtype=np.uint64)
        self.date_time = d0 + p.time_step * n
        self._solar, self._tick = sol, tick0 + n
        self._tod_prev, self._s_prev = flat[-4], flat[-2]
        self.current_od_temp = np.float64(tod)
        grid.current_signal = sig
        return TickWindow(buf)

    def _driver_window_loop(self, n_ticks: int) -> "TickWindow":
        p = self.init_props
        hp = p.cluster_prop.house_prop
        dts = p.time_step.seconds
        step = p.time_step
        solar_on, wa, shc = hp.solar_gain, hp.window_area, hp.shading_coeff
        tp, rng, grid = p.temp_prop, self.rng, self.power_grid
        date, tod, tick0 = self.date_time, self.current_od_temp, self._tick
        sol, s_prev = self._solar, self.power_grid.current_signal
        tods, sols, sprevs = [], [], []
        for _ in range(n_ticks):
            # environment.py:86-106: time advances, the cluster steps with the previous OD
            # temperature and the new datetime's solar gain, then a new OD temperature (1 gauss)
            # and the new signal; the reward of the tick uses the previous signal
            date = date + step
            sol = solar_gain(date, wa, shc) if solar_on else 0.0
            s_prev = grid.current_signal
            tods.append(tod)
            sols.append(sol)
            sprevs.append(s_prev)
            tod = od_temp(date, tp, rng)
            if grid.needs_state(dts):
                self._grid_pending = True
                break
            grid.step(date, tod, dts)
        k = len(tods)
        buf = np.empty((k, 4), np.float64)
        buf[:, 0] = tods
        buf[:, 1] = sols
        buf[:, 2] = sprevs
        buf[:, 3].view(np.uint64)[:] = np.arange(tick0, tick0 + k, dtype=np.uint64)
        self.date_time, self._solar, self._tick, self.current_od_temp = date, sol, tick0 + k, tod
        if k:
            self._tod_prev, self._s_prev = tods[-1], s_prev
        return TickWindow(buf)

    def finish_grid_step(self):
        """The grid step driver_window deferred (interpolation mode), once its ticks have run."""
        if self._grid_pending:
            self._grid_pending = False
            self.power_grid.step(self.date_time, self.current_od_temp, self.init_props.time_step.seconds)

    def _interp_evaluate(self, interp, ids, od, hour, date, factor) -> float:
        """Interpolated power of the sampled houses on device (k_interp_values; sharded: summed
        over ranks, one non-zero per slot, so exact), ordered sum x N/k (k_interp_sum)."""
        import torch

        sh = self._shard
        if getattr(sh, "_interp_src", None) is not interp.values:
            sh.interp_load(interp.grids, interp.values, interp.cfg)
            sh._interp_src = interp.values
        ids_t = torch.as_tensor(np.asarray(ids, np.int64)).to(sh.device)
        vals = torch.empty(len(ids), dtype=torch.float64, device=sh.device)
        sh.interp_values(ids_t, od, hour, date, vals)
        if self._comm is not None:
            self._comm.allreduce_sum(sh, vals)
        out = torch.empty(1, dtype=torch.float64, device=sh.device)
        sh.interp_sum(vals, factor, out)
        return float(out.item())

    def rollout(self, n_ticks: int, actions=None, action_mode: str = "random", rewards=None,
                use_graph: bool = False):
        """n_ticks steps in one C call.  ``actions``: uint8 [n_ticks, N] (buffer mode) or None;
        ``rewards``: float64 [n_ticks, N] output (allocated if None), or a 1-D [N] buffer that every
        tick overwrites.  Default (direct launches): the first window's count and its cluster power
        are launched before the host computes the drivers (mdr_rollout_begin), which then ride as
        kernel arguments of the first step kernel (k_step_window<..., KA>); the later windows'
        drivers are staged behind it.  ``use_graph=True``: the drivers are staged first and the
        launch sequence is replayed as a cached hipGraph (measured slower for both short and long
        calls, profiles/r02h_ab.log)."""
        import torch

        sh = self._shard
        if sh.penalty_mode != 0:
            raise NotImplementedError("rollout supports individual_L2; use step_tensor for common penalties")
        mode = ACTION_MODES[action_mode]
        if mode in (L.ACT_BANGBANG, L.ACT_DEADBAND_BANGBANG):
            raise NotImplementedError("bang-bang rollouts: use step_tensor(action_mode=..., lookahead=...)")
        if rewards is None:
            rewards = torch.empty((n_ticks, self._n_local), dtype=torch.float64, device=sh.device)
        rew_stride = 0 if rewards.dim() == 1 else self._n_local  # 1-D: every tick overwrites it
        drivers_whole = self.power_grid.interp is None and self._links is not None  # one driver window
        native = self._comm is not None and getattr(self._comm, "native", False)
        if (drivers_whole and not use_graph and (self._comm is None or native) and actions is None and n_ticks >= 2
                and self._vector_drivers_ok() and _host is not None and _host_gauss_ok(self.rng)
                and not self._grid_pending):
            # one C call: mdr_rollout_begin, the host drivers, mdr_rollout / mdr_rollout_sharded (no
            # Python between them: r06, the sharded call's Python driver loop cost ~50 us a call)
            launch = (L.fn_addr("mdr_rollout_begin"), L.fn_addr("mdr_rollout_sharded" if native else "mdr_rollout"),
                      sh.ctx.value, sh.stream(), rewards.data_ptr(), rew_stride, sh.p_dev.data_ptr(), mode,
                      1 if native else 0)
            ticks, launched = self._driver_window_vec(n_ticks, launch)
            if not launched:  # (the window crossed midnight: the drivers were finished in Python)
                if native:
                    self._comm.rollout(sh, ticks, None, mode, rewards, rew_stride)
                else:
                    sh.rollout(ticks, None, 0, mode, rewards, rew_stride, False)
            self._P_dev_valid = True
            self.finish_grid_step()
            self._counts_ready = 0
            return rewards
        if drivers_whole and not use_graph and (self._comm is None or getattr(self._comm, "native", False)):
            # the first window's count (sharded: + its allreduce) and P, before the drivers exist
            sh.rollout_begin(n_ticks, self._tick, actions, self._n_local if actions is not None else 0, mode)
        done = 0
        while done < n_ticks:  # one window unless interpolation ends it early (driver_window)
            ticks = self.driver_window(n_ticks - done)
            k = len(ticks)
            whole = done == 0 and k == n_ticks  # one window: the caller's buffers as they are
            a = None if actions is None else (actions if whole and actions.shape[0] == k else actions[done:done + k])
            r = rewards[done:done + k] if rew_stride and not (whole and rewards.shape[0] == k) else rewards
            if self._comm is not None:
                self._comm.rollout(sh, ticks, a, mode, r, rew_stride)
            else:
                # graphs are cached per (length, buffers): shorter windows only reuse them on 1-D rewards
                g = use_graph and (k == n_ticks or (a is None and not rew_stride))
                sh.rollout(ticks, a, self._n_local if a is not None else 0, mode, r, rew_stride, g)
            self._P_dev_valid = True
            self.finish_grid_step()
            done += k
        self._counts_ready = 0
        return rewards

    def greedy_rollout(self, n_ticks: int, actions=None, rewards=None):
        """Config C3's loop for n_ticks: ``greedy_actions`` then ``step_tensor(actions,
        ctrl='greedy_keys')`` every tick, as one C call per driver window (mdr_greedy_rollout: no
        Python between the ticks).  ``actions``: uint8 [n_ticks, N] (every tick's decisions) or a
        1-D [N] buffer every tick overwrites (allocated if None); ``rewards`` likewise (float64).
        Sharded, or a comm mode that draws per tick: the per-tick loop.  Returns (actions, rewards)."""
        import torch

        sh = self._shard
        n = self._n_local
        if actions is None:
            actions = torch.empty(n, dtype=torch.uint8, device=sh.device)
        if rewards is None:
            rewards = torch.empty((n_ticks, n), dtype=torch.float64, device=sh.device)
        for buf, dt, name in ((actions, torch.uint8, "actions"), (rewards, torch.float64, "rewards")):
            if buf.dtype != dt or buf.shape[-1] != n or not buf.is_contiguous() or buf.dim() not in (1, 2) or (
                    buf.dim() == 2 and buf.shape[0] < n_ticks):
                raise ValueError(f"{name}: a contiguous {dt} tensor [n_ticks, {n}] or [{n}]")
        a_st = n if actions.dim() == 2 else 0
        r_st = n if rewards.dim() == 2 else 0
        if (self.world > 1 or (self._gq_force_sharded and self._comm is not None) or self._links is None
                or self._grid_pending):
            for t in range(n_ticks):
                a = actions[t] if a_st else actions
                self.greedy_actions(out=a)
                self.step_tensor(a, rewards=rewards[t] if r_st else rewards, ctrl="greedy_keys")
            return actions, rewards
        done = 0
        while done < n_ticks:  # one window unless interpolation ends it early (driver_window)
            ticks = self.driver_window(n_ticks - done)
            k = len(ticks)
            sh.greedy_rollout(ticks, actions[done:] if a_st else actions, a_st,
                              rewards[done:] if r_st else rewards, r_st)
            self._P_dev_valid = True
            self.finish_grid_step()
            done += k
        self._counts_ready = 0
        return actions, rewards

    def greedy_actions(self, out=None):
        """GreedyMyopic.get_action (greedy_myopic_controller.py:67-104) on device: the next tick's
        actions from the current state, budget = the current regulation signal (obs reg_signal).
        Returns a uint8 [n_local] device tensor (``out`` if given).  Single shard: the launches also
        count the cluster power of these actions, so ``step_tensor(out)`` is one launch, and a
        preceding ``step_tensor(..., ctrl='greedy_keys')`` has already written their keys."""
        import torch

        sh = self._shard
        if out is None:
            out = torch.empty(self._n_local, dtype=torch.uint8, device=sh.device)
        if self.world > 1 or (self._gq_force_sharded and self._comm is not None):
            if self._hist_greedy_ok():
                # histogram select with the cluster's histograms: every rank
                # decides the same ≤ 4,096-house window, per-rank work O(N/G + window)
                S = float(self.power_grid.current_signal)
                v = sh.gq_shard_begin()
                self._comm.allreduce_count32(sh, v["super"])
                self._comm.allreduce_min(sh, v["range"])
                sh.gq_shard_bins(S)
                self._comm.allreduce_count32(sh, v["bins"])
                sh.gq_shard_compact(S, out)
                gathered = self._comm.allgather_bytes(sh, v["window"])
                sh.gq_shard_select(S, gathered, self.world, out)
                if not sh.gq_shard_fallback():
                    return out
                self._gq_shard_fallbacks += 1
            # the all-gather form (and the histogram form's fallback): all-gather this shard's
            # (key, P, lockout) rows in global order, the same selection on every rank, keep this
            # shard's slice
            nl = self._n_local
            key = torch.empty(nl, dtype=torch.float64, device=sh.device)
            pw = torch.empty(nl, dtype=torch.float64, device=sh.device)
            lk = torch.empty(nl, dtype=torch.uint8, device=sh.device)
            sh.greedy_inputs(key, pw, lk)
            sizes = [shard_range(self.n, r, self.world)[1] for r in range(self.world)]
            rows = [self._comm.allgather_cat(sh, t, sizes) for t in (key, pw, lk)]
            full = torch.empty(self.n, dtype=torch.uint8, device=sh.device)
            sh.greedy_select(self.n, *rows, float(self.power_grid.current_signal), full)
            out.copy_(full[self._offset:self._offset + nl])
            return out
        sh.greedy(float(self.power_grid.current_signal), out)
        self._counts_ready = ("greedy", out.data_ptr())
        return out

    def _hist_greedy_ok(self) -> bool:
        """The sharded histogram select applies: ≤ 4 capacity classes, ≤ 64 ranks, and a shard and
        comm that implement its stages."""
        return (self.world <= 64 and len(self._cap_values) <= 4 and hasattr(self._shard, "gq_shard_begin")
                and hasattr(self._comm, "allgather_bytes"))

    def rollout_stream(self):
        """Stream the step launches of ``rollout`` are issued on (for HIP-event timing)."""
        import torch

        return torch.cuda.current_stream(self._shard.device)

    # ------------------------------------------------------------------ observations
    def _cluster_power(self) -> float:
        if self._P_dev_valid:
            return float(self._shard.p_dev.item())
        return self._P_host

    def obs_spec(self):
        """mdr_obs_spec for the norm_state_dict layout of this config (norm.py:178-218)."""
        p = self.init_props
        cp, hp = p.cluster_prop, p.cluster_prop.house_prop
        sp, mp = p.state_prop, cp.message_prop
        links = self._obs_links
        if links is not None and not isinstance(links, np.ndarray):
            raise ValueError("ragged closed_groups neighbour lists (nb_comm < max_nb_agents_communication) "
                             "have no fixed-width observation vector")
        k = int(links.shape[1]) if links is not None else popmod.nb_comm(cp)
        msg_w = 4 + (4 if mp.thermal else 0) + (3 if mp.hvac else 0)
        n_feat = 10 + (2 if sp.hvac else 0) + (1 if sp.solar_gain else 0) + (5 if sp.thermal else 0) + k * msg_w
        spec = L.mdr_obs_spec()
        spec.n_feat = n_feat
        spec.hvac_state, spec.solar_state, spec.thermal_state = int(sp.hvac), int(sp.solar_gain), int(sp.thermal)
        spec.msg_thermal, spec.msg_hvac = int(mp.thermal), int(mp.hvac)
        spec.n_comm = k
        ring = cp.agents_comm_prop.mode == "neighbours"
        spec.comm_mode = L.COMM_RING if ring else L.COMM_TABLE
        spec.norm_reg_sig = float(p.reward_prop.norm_reg_sig)
        spec.cfg_ua, spec.cfg_ca, spec.cfg_cm, spec.cfg_hm = hp.Ua, hp.Ca, hp.Cm, hp.Hm
        spec.cfg_cap = float(hp.hvac_prop.cooling_capacity)
        return spec

    def bound_obs_spec(self):
        """(spec, scalars, keep): the obs spec with its device tables bound (comm table, ring halo
        of the neighbouring shards), the tick's obs scalars, and the tensors that must stay alive
        until the launch that reads them has run."""
        import torch

        sh = self._shard
        spec = self.obs_spec()
        keep = []
        if spec.comm_mode == L.COMM_TABLE and spec.n_comm > 0:
            links = np.asarray(self._obs_links, np.int32)
            if self.world > 1:
                # neighbours anywhere in the cluster: every shard's message rows, all-gathered in
                # global order (mdr_msg_pack), indexed by the global ids of this shard's table rows
                links = links[self._offset:self._offset + self._n_local]
                m = sh.lib.mdr_msg_width(L.C.byref(spec))
                mine = torch.empty((self._n_local, m), dtype=torch.float32, device=sh.device)
                sh.msg_pack(spec, mine)
                sizes = [shard_range(self.n, r, self.world)[1] * m for r in range(self.world)]
                allm = self._comm.allgather_cat(sh, mine.reshape(-1), sizes)
                keep.append(allm)
                spec.msg_all = L.ptr(allm)
            tab = torch.from_numpy(np.ascontiguousarray(links)).to(sh.device)
            keep.append(tab)
            spec.comm_table = L.ptr(tab)
        if spec.comm_mode == L.COMM_RING and self.world > 1 and spec.n_comm > 0:
            halo = self._comm.ring_halo(sh, spec)
            keep.append(halo)
            spec.halo_msg = L.ptr(halo)
        sc = L.mdr_obs_scalars(float(self._P_host), float(self.power_grid.current_signal),
                               float(self._solar), float(self.current_od_temp))
        return spec, sc, keep

    def obs_tensor(self, out=None):
        """``norm_state_dict`` for every local house as float32 [n_local, F] on device."""
        import torch

        sh = self._shard
        spec, sc, keep = self.bound_obs_spec()
        if out is None:
            out = torch.empty((self._n_local, spec.n_feat), dtype=torch.float32, device=sh.device)
        sh.obs(spec, sc, out, use_p_dev=self._P_dev_valid)
        if keep:
            torch.cuda.current_stream(sh.device).synchronize()
        return out

    def _params_host(self):
        if self._host_params is None:
            self._host_params = self._shard.host_params()
        return self._host_params

    def get_obs(self) -> Dict[int, dict]:
        """environment.py:110-130 — one 21-key dict per (local) house, with its messages.  Single
        shard: a LazyDict over a device snapshot of this tick's state, each house's dict built the
        first time it is read (one device->host copy on the first read).  Sharded: messages name
        houses on other shards, so the cluster state is gathered (a collective) and built now."""
        if self.world > 1:
            st, prm = self._comm.allgather_state(self._shard, self._shard.host_state(), self._params_host(), self.n)
            build = self._obs_builder(lambda: (st, prm), 0)
            return {g: build(g) for g in range(self._offset, self._offset + self._n_local)}
        sh = self._shard
        snap = (sh.t_air.clone(), sh.t_mass.clone(), sh.hvac.clone())
        cache = []

        def host():
            if not cache:
                from .shard import decode_hvac

                on, lock, sso = decode_hvac(snap[2].cpu().numpy())
                cache.append(({"T": snap[0].cpu().numpy(), "Tm": snap[1].cpu().numpy(), "on": on, "lock": lock,
                               "sso": sso}, self._params_host()))
            return cache[0]

        return LazyDict(self._obs_builder(host, 0), range(self._n_local))

    def _obs_builder(self, host, lo: int):
        """house id -> its obs dict, from the host arrays ``host()`` returns (state, params)
        indexed by global id, and this tick's scalars (captured now)."""
        p = self.init_props
        cp, hp = p.cluster_prop, p.cluster_prop.house_prop
        hv = hp.hvac_prop
        cap_values = list(self._cap_values)
        P, G = self._cluster_power(), self._solar
        od, dt_, S = self.current_od_temp, self.date_time, self.power_grid.current_signal
        L_, cop, lcf, db = hv.lockout_duration, hv.cop, hv.latent_cooling_fraction, hp.deadband
        mp = cp.message_prop
        links = self._obs_links

        def message(st, prm, j):
            cap = cap_values[int(prm["cap_idx"][j])]
            on_j = bool(st["on"][j])
            m = {"seconds_since_off": int(st["sso"][j]), "curr_consumption": cap / cop if on_j else 0.0,
                 "max_consumption": cap / cop, "lockout_duration": L_,
                 "current_temp_diff_to_target": float(st["T"][j]) - float(prm["target"][j])}
            if mp.hvac:
                m.update({"cop": cop, "latent_cooling_fraction": lcf, "cooling_capacity": cap})
            if mp.thermal:
                m.update({"Ca": float(prm["ca"][j]), "Ua": float(prm["ua"][j]), "Cm": float(prm["cm"][j]),
                          "Hm": float(prm["hm"][j])})
            return m

        def build(g):
            st, prm = host()
            row = links[g] if links is not None else ()
            return {
                "turned_on": bool(st["on"][g]), "seconds_since_off": int(st["sso"][g]), "lockout": bool(st["lock"][g]),
                "cop": cop, "cooling_capacity": cap_values[int(prm["cap_idx"][g])], "latent_cooling_fraction": lcf,
                "lockout_duration": L_, "target_temp": float(prm["target"][g]), "deadband": db,
                "Ua": float(prm["ua"][g]), "Ca": float(prm["ca"][g]), "Cm": float(prm["cm"][g]),
                "Hm": float(prm["hm"][g]), "indoor_temp": float(st["T"][g]), "mass_temp": float(st["Tm"][g]),
                "solar_gain": G, "cluster_hvac_power": P, "message": [message(st, prm, int(j)) for j in row],
                "OD_temp": od, "datetime": dt_, "reg_signal": S,
            }

        return build

    # ------------------------------------------------------------------ server-facing views
    def _building_views(self):
        """cluster.buildings: a lazy sequence of per-house views (built when indexed)."""
        return _BuildingList(self)

    # ------------------------------------------------------------------ checkpoint / deepcopy
    def state_dict(self) -> dict:
        sh = self._shard
        host = {k: getattr(sh, k).detach().cpu().clone() for k in
                ("t_air", "t_mass", "hvac", "ua", "ca", "cm", "hm", "target", "cap_idx")}
        host.update(date_time=self.date_time, current_od_temp=self.current_od_temp,
                    current_signal=self.power_grid.current_signal, solar=self._solar, tick=self._tick,
                    interp=None if self.power_grid.interp is None else
                    (self.power_grid.interp.since, self.power_grid.interp.base),
                    P=self._cluster_power(), cap_values=list(self._cap_values),
                    links=copy.deepcopy(self._links), obs_links=copy.deepcopy(self._obs_links))
        return host

    def load_state_dict(self, sd: dict) -> None:
        sh = self._shard
        if list(sd["cap_values"]) != list(self._cap_values):
            self._ensure_shard(sd["cap_values"])
            self._cap_values = list(sd["cap_values"])
            sh = self._shard
        for k in ("t_air", "t_mass", "hvac", "ua", "ca", "cm", "hm", "target", "cap_idx"):
            getattr(sh, k).copy_(sd[k].to(sh.device))
        sh.params_changed()
        self.date_time = sd["date_time"]
        self.current_od_temp = sd["current_od_temp"]
        self.power_grid.current_signal = sd["current_signal"]
        if sd.get("interp") is not None and self.power_grid.interp is not None:
            self.power_grid.interp.since, self.power_grid.interp.base = sd["interp"]
        self._solar, self._tick = sd["solar"], sd["tick"]
        self._P_host, self._P_dev_valid = sd["P"], False
        self._links = sd["links"]
        self._obs_links = sd["obs_links"]
        self._host_params = None
        self._counts_ready = 0

    def __deepcopy__(self, memo):
        """TrainingManager.test deep-copies the env (training_manager.py:269): clone the device
        state into a fresh context; the RNG is shared like the reference's global random."""
        new = object.__new__(Environment)
        memo[id(self)] = new
        # every nested reference to the RNG (the grid's Interpolator keeps one; by default it is
        # the `random` module, which deepcopy cannot copy) stays shared, like the reference's
        # global random
        memo[id(self.rng)] = self.rng
        for k, v in self.__dict__.items():
            if k in ("_shard", "cluster", "rng", "_comm", "_shard_factory"):
                continue
            new.__dict__[k] = copy.deepcopy(v, memo)
        new.rng, new._comm, new._shard_factory = self.rng, self._comm, self._shard_factory
        new.cluster = _ClusterView(new)
        new._shard = None
        new._ensure_shard(self._cap_values)
        new.load_state_dict(self.state_dict())
        return new
