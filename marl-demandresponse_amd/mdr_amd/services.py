"""The server's per-tick consumers of the environment, served from device reductions
(SURVEY §8(f) row 1).

The reference's services walk the N per-house observation dicts in Python every tick
(``Metrics.update`` loops over houses, ``ClientManagerService.update_data`` builds a pandas frame of
all of them).  Here every per-house quantity they need comes from ONE fused device reduction over
the state (``mdr_cluster_stats``, 12 sums/counts), so a tick costs O(1) host work at any N; the
per-house UI list is materialised only when read.

  DeviceMetrics  Metrics               server/app/services/metrics_service.py:71-257
  UISummary      ClientManagerService  server/app/services/client_manager_service.py:12-245
  ServerLoop     ControllerManager     server/app/services/controller_manager.py:93-260

Floating-point sums over houses are reduced in a fixed blocked order on the device, where the
reference adds house by house; they agree to rounding (tests/test_services_gpu.py: rtol 1e-12).
Reference quirks are kept: Metrics' ``indoor_temp - target_temp / nb_agents`` precedence, its
``cumul_squared_error_sig`` of the signal itself, ``cumul_squared_max_error_temp`` assigned (not
accumulated), the UI "Mass temperature" / "Target temperature" of house 0 only.
"""
from __future__ import annotations

from collections.abc import Sequence
from math import nan

import numpy as np

DESCRIPTION_KEYS = [
    "Number of HVAC",
    "Number of locked HVAC",
    "Outdoor temperature",
    "Average indoor temperature",
    "Average temperature difference",
    "Regulation signal",
    "Current consumption",
    "Consumption error (%)",
    "RMSE",
    "Mass temperature",
    "Target temperature",
    "Average temperature error",
]

# mdr_cluster_stats output slots (include/mdr.h)
S_TERR, S_ABS_TERR, S_MAX_TERR, S_SQ_TERR, S_REW, S_T, S_DIFF, S_ABS_DIFF, S_TM, S_TGT, S_LOCK, S_ON = range(12)


def cluster_stats(env, rewards=None) -> np.ndarray:
    """The 12 cluster statistics of the env's current state (+ ``rewards``, a device float64 [n_local]
    tensor, or None) as a host float64 array; sharded envs are reduced over ranks (sum, max)."""
    import torch

    sh = env.shard
    out = torch.empty(12, dtype=torch.float64, device=sh.device)
    sh.cluster_stats(rewards, out)
    if env.world > 1:
        comm = env._comm
        mx = out[S_MAX_TERR:S_MAX_TERR + 1].clone()
        out[S_MAX_TERR] = 0.0
        comm.allreduce_sum(sh, out)
        comm.allreduce_max(sh, mx)
        out[S_MAX_TERR] = mx[0]
    return out.cpu().numpy()


class DeviceMetrics:
    """``Metrics`` (metrics_service.py:71-257) fed by device reductions instead of a per-house loop."""

    FIELDS = ("cumul_avg_reward", "cumul_temp_offset", "cumul_temp_error", "cumul_signal_offset",
              "cumul_signal_error", "cumul_squared_error_temp", "max_temp_error", "cumul_OD_temp", "cumul_signal",
              "cumul_cons", "cumul_squared_error_sig", "cumul_squared_max_error_temp")

    def __init__(self, wandb_service=None):
        self.wandb_service = wandb_service

    def initialize(self, nb_agents: int, start_stats_from: int, nb_time_steps: int) -> None:
        self.nb_time_steps = nb_time_steps
        self.start_stats_from = start_stats_from
        self.nb_agents = nb_agents
        for f in self.FIELDS:
            setattr(self, f, 0.0)
        self.rmse_sig_per_ag = nan
        self.rmse_temp = nan
        self.rms_max_error_temp = nan
        if self.wandb_service is not None:
            self.wandb_service.initialize()

    def update(self, prev: dict, env, rewards, time_step: int) -> None:
        """Metrics.update(obs_dict, next_obs_dict, rewards_dict, time_step): ``prev`` holds the
        pre-step obs scalars {"reg_signal", "OD_temp", "cluster_hvac_power"} (observe(env) before
        the step); ``env`` is the post-step environment and ``rewards`` its device reward tensor."""
        n = self.nb_agents
        st = cluster_stats(env, rewards)
        self.cumul_temp_offset += st[S_TERR]
        self.cumul_temp_error += st[S_ABS_TERR]
        self.max_temp_error = max(self.max_temp_error, float(st[S_MAX_TERR]))
        self.cumul_avg_reward += st[S_REW]
        if time_step >= self.start_stats_from:
            self.cumul_squared_error_temp += st[S_SQ_TERR]
        # the same per-house signal error for every house (metrics_service.py:140-145)
        signal_error = (prev["reg_signal"] - env.cluster.current_power_consumption) / (n ** 2)
        self.cumul_signal_offset += n * signal_error
        self.cumul_signal_error += n * np.abs(signal_error)
        self.cumul_OD_temp += prev["OD_temp"]
        self.cumul_signal += prev["reg_signal"]
        self.cumul_cons += prev["cluster_hvac_power"]
        if time_step >= self.start_stats_from:
            self.cumul_squared_error_sig += prev["reg_signal"] ** 2
            self.cumul_squared_max_error_temp = self.max_temp_error ** 2

    def log(self, time_step: int, time_steps_log: int, time) -> dict:
        """Metrics.log without the reference's stray breakpoint (metrics_service.py:159-195)."""
        if time_step >= self.start_stats_from:
            self.update_rms(time_step)
        else:
            self.rmse_sig_per_ag = self.rmse_temp = self.rms_max_error_temp = nan
        metrics = {
            "Mean train return": self.cumul_avg_reward / time_steps_log,
            "Mean temperature offset": self.cumul_temp_offset / time_steps_log,
            "Mean temperature error": self.cumul_temp_error / time_steps_log,
            "Mean signal error": self.cumul_signal_offset / time_steps_log,
            "Mean signal offset": self.cumul_signal_offset / time_steps_log,
            "Mean outside temperature": self.cumul_OD_temp / time_steps_log,
            "Mean signal": self.cumul_signal / time_steps_log,
            "Mean consumption": self.cumul_cons / time_steps_log,
            "Time (hour)": time.hour,
            "Time step": time_step,
        }
        if self.wandb_service is not None:
            self.wandb_service.log(metrics)
        return metrics

    def reset(self) -> None:
        for f in ("cumul_avg_reward", "cumul_temp_offset", "cumul_temp_error", "max_temp_error",
                  "cumul_signal_offset", "cumul_signal_error", "cumul_OD_temp", "cumul_signal", "cumul_cons"):
            setattr(self, f, 0)

    def update_rms(self, time_step: int) -> None:
        k = time_step - self.start_stats_from
        self.rmse_sig_per_ag = np.sqrt(self.cumul_squared_error_sig / k) / self.nb_agents
        self.rmse_temp = np.sqrt(self.cumul_squared_error_temp / (k * self.nb_agents))
        self.rms_max_error_temp = np.sqrt(self.cumul_squared_max_error_temp / k)

    def update_final(self) -> dict:
        self.update_rms(self.nb_time_steps)
        return {"RMSE signal per agent": self.rmse_sig_per_ag, "RMSE temperature": self.rmse_temp,
                "RMS Max Error temperature": self.rms_max_error_temp}


def observe(env) -> dict:
    """The per-tick scalars every house's obs dict carries (environment.py:110-130)."""
    return {"reg_signal": env.power_grid.current_signal, "OD_temp": env.current_od_temp,
            "cluster_hvac_power": env.cluster.current_power_consumption}


class HouseList(Sequence):
    """ClientManagerService.update_houses_data's N-entry house list (client_manager_service.py:
    198-230) over a snapshot of the state: an entry is built when it is read.  The snapshot is a
    device copy until ``offload()`` moves it to host memory (UISummary keeps only the latest tick's
    list on the device, so a long server run grows host memory like the reference's list, not HBM)."""

    def __init__(self, env):
        sh = env.shard
        self._n = sh.n
        self._t, self._tg, self._hv = sh.t_air.clone(), sh.target.clone(), sh.hvac.clone()
        self._host = None
        self._lo = env._offset

    def _arrays(self):
        if self._host is None:
            from .shard import decode_hvac

            on, lock, sso = decode_hvac(self._hv.cpu().numpy())
            self._host = (self._t.cpu().numpy(), self._tg.cpu().numpy(), on, lock, sso)
            self._t = self._tg = self._hv = None  # (the device copies are no longer needed)
        return self._host

    def offload(self) -> None:
        """Move the snapshot to host memory now (one device->host copy) and free its device copy."""
        self._arrays()

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        T, tg, on, lock, sso = self._arrays()
        i = int(i)
        if i < 0:
            i += len(self)
        d = {"id": self._lo + i}
        if on[i]:
            d["hvacStatus"] = "ON"
        else:
            d.update({"hvacStatus": "Lockout" if lock[i] else "OFF", "secondsSinceOff": int(sso[i])})
        d["indoorTemp"] = float(T[i])
        d["targetTemp"] = float(tg[i])
        d["tempDifference"] = float(T[i]) - float(tg[i])
        return d

    def status_counts(self):
        """(#ON, #Lockout, #OFF, sum of secondsSinceOff over the non-ON houses)."""
        _, _, on, lock, sso = self._arrays()
        off = ~on
        return int(on.sum()), int((off & lock).sum()), int((off & ~lock).sum()), int(sso[off].sum())


class UISummary:
    """ClientManagerService (client_manager_service.py:28-245) from device reductions: the 12
    summary strings, the graph series and the house list of every tick, without a pandas frame."""

    def __init__(self, socket_manager=None):
        self.socket_manager = socket_manager

    def initialize_data(self, interface: bool) -> None:
        self.interface = interface
        self.description = {}
        self.temp_diff = np.array([])
        self.temp_err = np.array([])
        self.air_temp = np.array([])
        self.mass_temp = np.array([])
        self.target_temp = np.array([])
        self.outdoor_temp = np.array([])
        self.signal = np.array([])
        self.consumption = np.array([])
        self.houses_data = {}

    def update_data(self, env, time_step: int) -> None:
        """update_data(obs_dict, time_step) for the env's current obs."""
        n = env.n
        st = cluster_stats(env)
        od, S, P = env.current_od_temp, env.power_grid.current_signal, env.cluster.current_power_consumption
        # update_graph_data (client_manager_service.py:177-196): per-tick means over the houses
        self.temp_diff = np.append(self.temp_diff, st[S_DIFF] / n)
        self.temp_err = np.append(self.temp_err, st[S_ABS_DIFF] / n)
        self.air_temp = np.append(self.air_temp, st[S_T] / n)
        self.mass_temp = np.append(self.mass_temp, st[S_TM] / n)
        self.target_temp = np.append(self.target_temp, st[S_TGT] / n)
        self.outdoor_temp = np.append(self.outdoor_temp, od)
        self.signal = np.append(self.signal, S)
        self.consumption = np.append(self.consumption, P)
        tm0, tg0 = self._house0(env)
        values = [
            str(n),
            str(int(st[S_LOCK])),
            str(round(od, 2)),
            str(round(st[S_T] / n, 2)),
            str(round(st[S_DIFF] / n, 2)),
            str(S),
            str(P),
            str((S - P) / S * 100),
            str(np.sqrt(np.mean((self.signal - self.consumption) ** 2))),
            str(round(tm0, 2)),
            str(round(tg0, 2)),
            str(np.mean(self.temp_err)),
        ]
        self.description[time_step] = dict(zip(DESCRIPTION_KEYS, values))
        if self.houses_data:  # the previous tick's snapshot leaves HBM
            self.houses_data[next(reversed(self.houses_data))].offload()
        self.houses_data[time_step] = HouseList(env)

    @staticmethod
    def _house0(env):
        """mass_temp / target_temp of house 0 (the reference reads data_frame[...][0])."""
        import torch

        sh = env.shard
        v = torch.stack([sh.t_mass[0], sh.target[0]]) if env._offset == 0 else \
            torch.zeros(2, dtype=torch.float64, device=sh.device)
        if env.world > 1:
            env._comm.allreduce_sum(sh, v)
        a, b = v.cpu().tolist()
        return a, b


class ServerLoop:
    """ControllerManager.start's tick loop (controller_manager.py:129-187) on the device env:
    UI summary of the current obs -> actions -> env.step -> Metrics.update -> episode reset ->
    periodic log.  ``controller``: 'deadband_bangbang' / 'bangbang' / 'always_on' / 'random' (fused
    in the step kernel), 'greedy' (device GreedyMyopic), or a callable env -> uint8 device actions.
    Per-house Python objects are only built on access (UISummary.houses_data)."""

    def __init__(self, env, controller="deadband_bangbang", start_stats_from: int = 0, nb_time_steps: int = 1000,
                 time_steps_per_episode: int = 10 ** 9, time_steps_train_log: int = 10 ** 9, interface: bool = False,
                 metrics=None, ui=None):
        self.env = env
        self.controller = controller
        self.metrics = metrics or DeviceMetrics()
        self.ui = ui or UISummary()
        self.metrics.initialize(env.n, start_stats_from, nb_time_steps)
        self.ui.initialize_data(interface)
        self.nb_time_steps = nb_time_steps
        self.time_steps_per_episode = time_steps_per_episode
        self.time_steps_train_log = time_steps_train_log
        self.current_time_step = 0
        self.logs = []

    def _step(self):
        env, c = self.env, self.controller
        if callable(c):
            return env.step_tensor(c(env))
        if c == "greedy":
            return env.step_tensor(env.greedy_actions())
        if c in ("deadband_bangbang", "bangbang", "always_on", "random"):
            # the launch also counts the next tick's power under the same source (one launch per tick)
            return env.step_tensor(None, action_mode=c, lookahead=c)
        raise ValueError(f"unknown controller {c!r}")

    def run(self, n_steps=None):
        end = self.nb_time_steps if n_steps is None else min(self.nb_time_steps, self.current_time_step + n_steps)
        for step in range(self.current_time_step, end):
            self.ui.update_data(self.env, step)
            prev = observe(self.env)
            rewards = self._step()
            self.metrics.update(prev, self.env, rewards, step)
            if step % self.time_steps_per_episode == self.time_steps_per_episode - 1:
                self.env.reset(return_obs=False)
            if step % self.time_steps_train_log == self.time_steps_train_log - 1:
                self.logs.append(self.metrics.log(step, self.time_steps_train_log, self.env.date_time))
                self.metrics.reset()
            self.current_time_step += 1
        if self.current_time_step == self.nb_time_steps:
            return self.metrics.update_final()
        return None
