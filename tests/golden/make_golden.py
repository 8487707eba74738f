"""Generate the golden parity fixtures by running the REFERENCE env core in this container.

This script is the only place that imports the reference (read-only, /root/reference).  It runs
here, never on the GPU box; only its outputs (``tests/golden/*.npz``, ``*.json``) travel.  The
fixtures are data: inputs and the reference's outputs for them.

Recipe:
  * ``PYTHONPATH=<stubdir>:/root/reference/server``, ``TZ=UTC``;
  * ``<stubdir>/perlin_noise`` is an import-only stub whose ``noise()`` raises, so perlin mode can
    never silently produce a fixture (perlin parity is unpinned);
  * three ``sys.modules`` shims let the controller modules import without the server stack
    (``app.core.agents.controllers`` package init pulls cvxpy/v0; ``parser_service`` and
    ``app.utils.logger`` pull pydantic-v1 ``BaseSettings``).

Fixtures (names follow SURVEY §8(c) F1..F9):
  F1 lockout.npz       HVAC.step sequences, L in {12, 40}, dt in {4, 3}, random action strings
  F2 thermal.npz       Building.update_temperature over a random grid (Ua ~1 and 218, on/off, dt)
  F3 solar.npz         compute_solar_gain over a (month, day, hour, minute) sweep
  F4 signal.npz        flat / sinusoidals / regular_steps signals over a datetime sweep
  F5 rewards.npz       RewardsCalculator in all 4 penalty modes
  F6 traj_*.npz        seeded end-to-end trajectories (Environment.reset/step + norm_state_dict)
  F7 greedy.npz        GreedyMyopic decisions along a trajectory
  F8 comm.json         neighbour tables for the deterministic comm modes (+ random_fixed seeded)
  F9 rng_order.npz     population after 1 and 3 resets for seeds {0, 4, 123}
  P  policy.npz        MAPPO actor (seed 1, the reference init) on reference norm_state_dict
                       vectors: weights, obs, Actor.forward probabilities (row P)
  f1 services.npz     reference Metrics + ClientManagerService along a ControllerManager loop
  f2 mappo.npz        one reference MAPPO.update at N = 2 (init, transitions, returns, final weights)
  a10 interp.npz       PowerInterpolator.interpolate_grid_fast on 400 swept points over a synthetic
                       table of the reference grid (interp_parameters_dict.json / interp_dict_keys.csv,
                       copied next to it), + traj_interp_*.npz trajectories in interpolation mode

Usage:  python tests/golden/make_golden.py   (writes next to this file)
"""
from __future__ import annotations

import copy
import datetime as dt
import json
import os
import random
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference/server"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs() -> None:
    os.environ["TZ"] = "UTC"
    os.environ.setdefault("MPLBACKEND", "Agg")
    stub = tempfile.mkdtemp(prefix="mdr_refstub_")
    os.makedirs(os.path.join(stub, "perlin_noise"))
    with open(os.path.join(stub, "perlin_noise", "__init__.py"), "w") as f:
        f.write(
            "class PerlinNoise:\n"
            "    def __init__(self, octaves=1, seed=None):\n"
            "        self.octaves, self.seed = octaves, seed\n"
            "    def noise(self, *a, **k):\n"
            "        raise RuntimeError('perlin_noise is absent: perlin parity is unpinned')\n"
        )
    sys.path[:0] = [stub, REF]
    import logging

    lg = types.ModuleType("app.utils.logger")
    lg.logger = logging.getLogger("ref")
    sys.modules["app.utils.logger"] = lg
    ps = types.ModuleType("app.services.parser_service")
    ps.MarlConfig = object
    sys.modules["app.services.parser_service"] = ps
    ctl = types.ModuleType("app.core.agents.controllers")
    ctl.__path__ = [os.path.join(REF, "app/core/agents/controllers")]
    sys.modules["app.core.agents.controllers"] = ctl
    # services (Metrics, ClientManagerService) without wandb / socket.io: no-op stand-ins
    wb = types.ModuleType("app.services.wandb_service")

    class WandbManager:
        def initialize(self, *a, **k):
            pass

        def log(self, *a, **k):
            pass

        def save(self, *a, **k):
            pass

    wb.WandbManager = WandbManager
    sys.modules["app.services.wandb_service"] = wb
    sm = types.ModuleType("app.services.socket_manager_service")
    sm.SocketManager = object
    sys.modules["app.services.socket_manager_service"] = sm


_install_stubs()

from app.core.environment.environment import Environment  # noqa: E402
from app.core.environment.environment_properties import EnvironmentProperties  # noqa: E402
from app.core.environment.cluster.hvac import HVAC  # noqa: E402
from app.core.environment.cluster.building import Building  # noqa: E402
from app.core.environment.environment_properties import (  # noqa: E402
    BuildingProperties,
    HvacProperties,
    RewardProperties,
)
from app.core.environment.power_grid.signal_calculator import SignalCalculator  # noqa: E402
from app.core.environment.power_grid.power_grid_properties import SignalProperties  # noqa: E402
from app.core.environment.rewards_calculator import RewardsCalculator  # noqa: E402
from app.core.environment.cluster.agent_communication_builder import (  # noqa: E402
    AgentCommunicationBuilder,
)
from app.core.environment.cluster.cluster_properties import (  # noqa: E402
    AgentsCommunicationProperties,
)
from app.utils.utils import compute_solar_gain  # noqa: E402
from app.utils.norm import norm_state_dict  # noqa: E402
from app.core.agents.controllers.bangbang_controllers import (  # noqa: E402
    DeadbandBangBangController,
    BangBangController,
)
from app.core.agents.controllers import greedy_myopic_controller as greedy_mod  # noqa: E402

MARL_JSON = os.path.join(REF, "app/core/config/MARLconfig.json")


def env_prop_json() -> dict:
    with open(MARL_JSON) as f:
        return json.load(f)["env_prop"]


def make_props(overrides: dict) -> EnvironmentProperties:
    d = copy.deepcopy(env_prop_json())
    for path, val in overrides.items():
        cur = d
        keys = path.split(".")
        for k in keys[:-1]:
            cur = cur[k]
        cur[keys[-1]] = val
    return EnvironmentProperties.parse_obj(d)


def epoch(t: dt.datetime) -> float:
    return (t - dt.datetime(1970, 1, 1)).total_seconds()


# ---------------------------------------------------------------------------------------- F1
def gen_lockout() -> None:
    rs = np.random.RandomState(11)
    out = {}
    cases = [(12, 4), (40, 4), (40, 3), (10, 4)]
    for ci, (L, step) in enumerate(cases):
        hv = HVAC(HvacProperties(lockout_duration=L))
        T = 300
        acts = rs.randint(0, 2, size=T).astype(np.uint8)
        # bias some strings toward long on / off runs
        if ci % 2 == 1:
            acts = np.repeat(rs.randint(0, 2, size=T // 10), 10).astype(np.uint8)
        on = np.zeros(T, np.uint8)
        lock = np.zeros(T, np.uint8)
        sso = np.zeros(T, np.int64)
        for t in range(T):
            hv.step(bool(acts[t]), dt.timedelta(seconds=step))
            on[t], lock[t], sso[t] = bool(hv.turned_on), bool(hv.lockout), hv.seconds_since_off
        out[f"c{ci}_L"] = np.int64(L)
        out[f"c{ci}_dt"] = np.int64(step)
        out[f"c{ci}_action"] = acts
        out[f"c{ci}_on"] = on
        out[f"c{ci}_lock"] = lock
        out[f"c{ci}_sso"] = sso
    out["ncases"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(OUT, "lockout.npz"), **out)


# ---------------------------------------------------------------------------------------- F2
def gen_thermal() -> None:
    rs = np.random.RandomState(12)
    M = 600
    cols = {k: np.zeros(M) for k in
            ("Ua", "Ca", "Cm", "Hm", "T", "Tm", "Tod", "cap", "solar_gain", "T_new", "Tm_new")}
    on = np.zeros(M, np.uint8)
    step = np.zeros(M, np.int64)
    stamp = np.zeros(M, np.float64)
    solar_flag = np.zeros(M, np.uint8)
    base = dt.datetime(2021, 1, 1)
    for i in range(M):
        bp = BuildingProperties()
        b = Building(bp)
        ua = rs.uniform(0.9, 1.1) if i % 2 == 0 else 218.0 * rs.uniform(0.9, 1.1)
        b.init_props.Ua = ua
        b.init_props.Ca = 9.08e5 * rs.uniform(0.9, 1.1)
        b.init_props.Cm = 3.45e6 * rs.uniform(0.9, 1.1)
        b.init_props.Hm = 2.84e3 * rs.uniform(0.9, 1.1)
        b.init_props.solar_gain = bool(i % 5 != 4)
        b.indoor_temp = rs.uniform(10, 35)
        b.current_mass_temp = rs.uniform(10, 35)
        b.hvac.turned_on = bool(rs.randint(0, 2))
        b.hvac.init_props.cooling_capacity = float(rs.choice([12500, 15000, 17500]))
        s = int(rs.choice([1, 4, 4, 4, 60]))
        when = base + dt.timedelta(days=int(rs.randint(0, 364)), seconds=int(rs.randint(0, 86400)))
        tod = rs.uniform(10, 40)
        cols["Ua"][i], cols["Ca"][i] = b.init_props.Ua, b.init_props.Ca
        cols["Cm"][i], cols["Hm"][i] = b.init_props.Cm, b.init_props.Hm
        cols["T"][i], cols["Tm"][i], cols["Tod"][i] = b.indoor_temp, b.current_mass_temp, tod
        cols["cap"][i] = b.hvac.init_props.cooling_capacity
        on[i], step[i], stamp[i] = b.hvac.turned_on, s, epoch(when)
        solar_flag[i] = b.init_props.solar_gain
        b.update_temperature(tod, dt.timedelta(seconds=s), when)
        cols["T_new"][i], cols["Tm_new"][i] = b.indoor_temp, b.current_mass_temp
        cols["solar_gain"][i] = b.current_solar_gain
    np.savez_compressed(os.path.join(OUT, "thermal.npz"), on=on, dt=step, epoch=stamp,
                        solar_flag=solar_flag, **cols)


# ---------------------------------------------------------------------------------------- F3
def gen_solar() -> None:
    stamps, vals = [], []
    for month in range(1, 13):
        for day in (1, 9, 15, 28):
            for minute_of_day in range(0, 24 * 60, 7):
                t = dt.datetime(2021, month, day, minute_of_day // 60, minute_of_day % 60)
                stamps.append(epoch(t))
                vals.append(compute_solar_gain(t, 7.175, 0.67))
    np.savez_compressed(os.path.join(OUT, "solar.npz"), epoch=np.array(stamps),
                        gain=np.array(vals, np.float64))


# ---------------------------------------------------------------------------------------- F4
def gen_signal() -> None:
    out = {}
    t0 = dt.datetime(2021, 3, 7, 0, 0, 0)
    stamps = [t0 + dt.timedelta(seconds=4 * k + (k % 7)) for k in range(0, 24 * 900, 9)]
    out["epoch"] = np.array([epoch(t) for t in stamps])
    for mode in ("flat", "sinusoidals", "regular_steps"):
        for nb in (50, 1000):
            sp = SignalProperties(mode=mode)
            sc = SignalCalculator(sp, nb)
            base = 4200.0 * nb
            out[f"{mode}_{nb}"] = np.array([float(sc.compute_signal(base, t)) for t in stamps])
    # non-default amplitude / period settings
    sp = SignalProperties(mode="sinusoidals", amplitude_ratios=[0.2, 0.05, 0.1],
                          periods=[300, 900, 3600])
    sc = SignalCalculator(sp, 77)
    out["sinusoidals_custom_77"] = np.array([float(sc.compute_signal(77 * 3900.0, t)) for t in stamps])
    sp = SignalProperties(mode="regular_steps", amplitude_per_hvac=5000, period=600)
    sc = SignalCalculator(sp, 77)
    out["regular_steps_custom_77"] = np.array([float(sc.compute_signal(77 * 3900.0, t)) for t in stamps])
    np.savez_compressed(os.path.join(OUT, "signal.npz"), **out)


# ---------------------------------------------------------------------------------------- F5
def gen_rewards() -> None:
    rs = np.random.RandomState(15)
    out = {}
    N = 8
    bp = BuildingProperties(target_temp=19.0, deadband=0.5)
    buildings = []
    for i in range(N):
        b = Building(bp)
        b.init_props.target_temp = 19.0 + abs(rs.normal())
        b.indoor_temp = rs.uniform(16, 24)
        buildings.append(b)
    out["target"] = np.array([b.init_props.target_temp for b in buildings])
    out["T"] = np.array([b.indoor_temp for b in buildings])
    out["deadband"] = np.float64(0.5)
    out["P"] = np.float64(41000.0)
    out["S"] = np.float64(36517.25)
    for mode in ("individual_L2", "common_L2", "common_max_error", "mixture"):
        rp = RewardProperties()
        rp.penalty_props.mode = mode
        rp.penalty_props.alpha_common_max = 0.5 if mode == "mixture" else 0.0
        rc = RewardsCalculator(rp, bp)
        r = rc.compute_rewards(buildings, 41000.0, 36517.25)
        out[f"reward_{mode}"] = np.array([r[i] for i in range(N)])
    np.savez_compressed(os.path.join(OUT, "rewards.npz"), **out)


# ---------------------------------------------------------------------------------------- F6
POP_KEYS = ("Ua", "Ca", "Cm", "Hm", "target_temp", "cooling_capacity")


def population(env) -> dict:
    bs = env.cluster.buildings
    return {
        "Ua": np.array([b.init_props.Ua for b in bs]),
        "Ca": np.array([b.init_props.Ca for b in bs]),
        "Cm": np.array([b.init_props.Cm for b in bs]),
        "Hm": np.array([b.init_props.Hm for b in bs]),
        "target_temp": np.array([b.init_props.target_temp for b in bs]),
        "cooling_capacity": np.array([float(b.hvac.init_props.cooling_capacity) for b in bs]),
        "init_air_temp_noised": np.array([b.init_props.init_air_temp for b in bs]),
    }


def record_obs(obs: dict, N: int) -> dict:
    o = [obs[i] for i in range(N)]
    return {
        "T": np.array([x["indoor_temp"] for x in o], np.float64),
        "Tm": np.array([x["mass_temp"] for x in o], np.float64),
        "on": np.array([bool(x["turned_on"]) for x in o], np.uint8),
        "lock": np.array([bool(x["lockout"]) for x in o], np.uint8),
        "sso": np.array([x["seconds_since_off"] for x in o], np.int64),
        "P": np.float64(o[0]["cluster_hvac_power"]),
        "S": np.float64(o[0]["reg_signal"]),
        "Tod": np.float64(o[0]["OD_temp"]),
        "G": np.float64(o[0]["solar_gain"]),
        "epoch": np.float64(epoch(o[0]["datetime"])),
        # one neighbour message per house, first in comm order (checks message fields)
        "msg0_diff": np.array([x["message"][0]["current_temp_diff_to_target"] if x["message"] else 0.0
                               for x in o], np.float64),
        "msg0_curr": np.array([x["message"][0]["curr_consumption"] if x["message"] else 0.0
                               for x in o], np.float64),
    }


def gen_traj(name: str, overrides: dict, N: int, T: int, seed: int, controller: str,
             norm_ticks=(0, 1, 2, 50), resets: int = 3, action_seed: int = 1234) -> None:
    overrides = dict(overrides)
    overrides["cluster_prop.nb_agents"] = N
    props = make_props(overrides)
    random.seed(seed)
    env = Environment(props)
    obs = None
    for _ in range(resets - 1):
        obs = env.reset()
    if obs is None:
        obs = env.get_obs()
    pop = population(env)
    rs = np.random.RandomState(action_seed)
    if controller == "random":
        actions = rs.randint(0, 2, size=(T, N)).astype(np.uint8)
    else:
        actions = np.zeros((T, N), np.uint8)
    ctl = None
    if controller == "deadband_bbc":
        ctl = [DeadbandBangBangController({"id": i}, None) for i in range(N)]
    elif controller == "bbc":
        ctl = [BangBangController({"id": i}, None) for i in range(N)]
    rec = {k: [] for k in record_obs(obs, N)}
    rec["reward"] = []
    o0 = record_obs(obs, N)
    norms = {}
    if 0 in norm_ticks:
        norms["norm_t0"] = np.array(norm_state_dict(obs, env.init_props))
    for t in range(T):
        if ctl is not None:
            a = {i: ctl[i].act(obs) for i in range(N)}
            actions[t] = [bool(a[i]) for i in range(N)]
        else:
            a = {i: bool(actions[t, i]) for i in range(N)}
        obs, rew = env.step(a)
        r = record_obs(obs, N)
        for k, v in r.items():
            rec[k].append(v)
        rec["reward"].append(np.array([rew[i] for i in range(N)], np.float64))
        if (t + 1) in norm_ticks:
            norms[f"norm_t{t + 1}"] = np.array(norm_state_dict(obs, env.init_props))
    out = {f"pop_{k}": v for k, v in pop.items()}
    out.update({f"init_{k}": v for k, v in o0.items()})
    out.update({f"traj_{k}": np.stack(v) if np.ndim(v[0]) else np.array(v) for k, v in rec.items()})
    out.update(norms)
    out["actions"] = actions
    out["N"], out["T"], out["seed"], out["resets"] = np.int64(N), np.int64(T), np.int64(seed), np.int64(resets)
    meta = {"overrides": overrides, "controller": controller, "N": N, "T": T, "seed": seed,
            "resets": resets, "action_seed": action_seed, "norm_ticks": list(norm_ticks)}
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(OUT, f"traj_{name}.npz"), **out)


# ---------------------------------------------------------------------------------------- F7
def gen_greedy() -> None:
    N, T = 120, 25
    props = make_props({"cluster_prop.nb_agents": N,
                        "power_grid_prop.signal_properties.mode": "sinusoidals"})
    random.seed(7)
    env = Environment(props)
    obs = env.reset()
    greedy_mod.global_myopic_memory[0] = None
    greedy_mod.global_myopic_memory[1] = None
    ctl = [greedy_mod.GreedyMyopic({"id": i}, None) for i in range(N)]
    rec = {"T": [], "target": [], "cap": [], "lock": [], "S": [], "action": []}
    for t in range(T):
        a = {i: int(ctl[i].act(obs)) for i in range(N)}
        rec["T"].append([obs[i]["indoor_temp"] for i in range(N)])
        rec["target"].append([obs[i]["target_temp"] for i in range(N)])
        rec["cap"].append([float(obs[i]["cooling_capacity"]) for i in range(N)])
        rec["lock"].append([bool(obs[i]["lockout"]) for i in range(N)])
        rec["S"].append(float(obs[0]["reg_signal"]))
        rec["action"].append([a[i] for i in range(N)])
        obs, _ = env.step(a)
    out = {k: np.array(v) for k, v in rec.items()}
    out["cop"] = np.float64(2.5)
    np.savez_compressed(os.path.join(OUT, "greedy.npz"), **out)


# ---------------------------------------------------------------------------------------- F8
def gen_comm() -> None:
    out = {}
    for mode, ns in (("neighbours", (2, 3, 7, 11, 50)), ("closed_groups", (7, 11, 25, 50, 53)),
                     ("neighbours_2D", (25, 50, 100))):
        for n in ns:
            for kmax in (10, 4):
                p = AgentsCommunicationProperties(mode=mode, max_nb_agents_communication=kmax,
                                                  row_size=5 if n != 100 else 10,
                                                  max_communication_distance=2 if n != 25 else 1)
                try:
                    links = AgentCommunicationBuilder(p, n).get_comm_link_list()
                    out[f"{mode}_{n}_{kmax}"] = [[int(j) for j in links[i]] for i in range(n)]
                except ValueError as e:
                    out[f"{mode}_{n}_{kmax}"] = "ValueError: " + str(e)
    random.seed(99)
    p = AgentsCommunicationProperties(mode="random_fixed", max_nb_agents_communication=4)
    links = AgentCommunicationBuilder(p, 12).get_comm_link_list()
    out["random_fixed_12_4_seed99"] = [[int(j) for j in links[i]] for i in range(12)]
    with open(os.path.join(OUT, "comm.json"), "w") as f:
        json.dump(out, f)


# ---------------------------------------------------------------------------------------- F9
def gen_rng_order() -> None:
    out = {}
    for seed in (0, 4, 123):
        for mode in ("random", "fixed"):
            props = make_props({"cluster_prop.nb_agents": 20, "start_datetime_mode": mode,
                                "power_grid_prop.signal_properties.mode": "flat"})
            random.seed(seed)
            env = Environment(props)
            p1 = population(env)
            e1 = epoch(env.date_time)
            env.reset()
            env.reset()
            p3 = population(env)
            e3 = epoch(env.date_time)
            for k, v in p1.items():
                out[f"s{seed}_{mode}_r1_{k}"] = v
            for k, v in p3.items():
                out[f"s{seed}_{mode}_r3_{k}"] = v
            out[f"s{seed}_{mode}_r1_epoch"] = np.float64(e1)
            out[f"s{seed}_{mode}_r3_epoch"] = np.float64(e3)
            out[f"s{seed}_{mode}_r3_Tod"] = np.float64(env.current_od_temp)
            out[f"s{seed}_{mode}_r3_next_random"] = np.float64(random.random())
    np.savez_compressed(os.path.join(OUT, "rng_order.npz"), **out)


# ---------------------------------------------------------------------------------------- P
def gen_policy() -> None:
    """MAPPO(MAPPOProperties(), num_state=F, seed=1) (mappo.py:37-60) on the norm_state_dict vectors
    the trajectory fixtures hold; probabilities from its actor_net (network.py:29-33) in fp32."""
    import torch

    from app.core.agents.trainables.mappo import MAPPO, MAPPOProperties

    out = {}
    for case, (traj, keys) in {"c1": ("c1_sin_dbbc", ("norm_t0", "norm_t1", "norm_t50")),
                               "wide": ("n30_maxerr_groups_hvacmsg", ("norm_t0", "norm_t50"))}.items():
        d = np.load(os.path.join(OUT, f"traj_{traj}.npz"))
        obs = np.concatenate([d[k] for k in keys]).astype(np.float32)
        agent = MAPPO(MAPPOProperties(), num_state=obs.shape[1])
        with torch.no_grad():
            probs = agent.actor_net(torch.from_numpy(obs)).numpy()
        for k, v in agent.actor_net.state_dict().items():
            out[f"{case}_{k}"] = v.numpy()
        out[f"{case}_obs"] = obs
        out[f"{case}_probs"] = probs
        # select_actions on the same vectors: last_probs[i] = probs[i, action[i]]
        torch.manual_seed(7)
        acts = agent.select_actions(list(obs.astype(np.float64)))
        out[f"{case}_sel_action"] = np.array([acts[i] for i in range(len(obs))], np.int64)
        out[f"{case}_sel_prob"] = np.array([agent.last_probs[i] for i in range(len(obs))], np.float32)
    np.savez_compressed(os.path.join(OUT, "policy.npz"), **out)


# ---------------------------------------------------------------------------------------- a10
INTERP_SRC = os.path.join(REF, "v0/monteCarlo")
INTERP_SEED = 2024
BPP = "power_grid_prop.base_power_props."


def interp_table_path() -> str:
    """The synthetic Monte-Carlo table (oracle/interp_np.synthetic_table, seed 2024) as a .npy
    (the reference does not ship mergedGridSearchResultFinal.npy); tests rebuild the same file."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from oracle.interp_np import synthetic_table

    with open(os.path.join(OUT, "interp_parameters_dict.json")) as f:
        params = json.load(f)
    path = os.path.join(tempfile.gettempdir(), f"mdr_interp_table_{INTERP_SEED}.npy")
    np.save(path, synthetic_table([len(v) for v in params.values()], INTERP_SEED))
    return path


def interp_overrides(extra: dict) -> dict:
    d = {BPP + "mode": "interpolation", BPP + "path_datafile": interp_table_path(),
         BPP + "path_parameter_dict": os.path.join(OUT, "interp_parameters_dict.json"),
         BPP + "path_dict_keys": os.path.join(OUT, "interp_dict_keys.csv")}
    d.update(extra)
    return d


def gen_interp() -> None:
    """a10: PowerInterpolator.interpolate_grid_fast on swept points (inside, outside and exactly
    on the grid) of the reference grid over the synthetic table."""
    import shutil

    from app.core.environment.power_grid.interpolation import PowerInterpolator
    from app.core.environment.power_grid.power_grid_properties import BasePowerProperties

    for name in ("interp_parameters_dict.json", "interp_dict_keys.csv"):
        shutil.copy(os.path.join(INTERP_SRC, name), os.path.join(OUT, name))
    bpp = BasePowerProperties(mode="interpolation", path_datafile=interp_table_path(),
                              path_parameter_dict=os.path.join(OUT, "interp_parameters_dict.json"),
                              path_dict_keys=os.path.join(OUT, "interp_dict_keys.csv"))
    pi = PowerInterpolator(bpp, BuildingProperties())
    keys = list(pi.dict_keys)
    rs = np.random.RandomState(21)
    M = 400
    raw, clipped, val = np.zeros((M, len(keys))), np.zeros((M, len(keys))), np.zeros(M)
    for m in range(M):
        pt = {}
        for k in keys:
            g = np.array(pi.parameters_dict[k], np.float64)
            lo, hi = g.min(), g.max()
            if m % 4 == 0 or rs.random_sample() < 0.15:
                pt[k] = float(rs.choice(g))  # exactly on a grid point (the ends included)
            else:
                pt[k] = float(rs.uniform(lo - 0.15 * (hi - lo), hi + 0.15 * (hi - lo)))
        raw[m] = [pt[k] for k in keys]
        pt = pi.clip_interpolation_point(pt)
        clipped[m] = [pt[k] for k in keys]
        val[m] = float(pi.interpolate_grid_fast(pt))
    np.savez_compressed(os.path.join(OUT, "interp.npz"), keys=np.array(keys), raw=raw, clipped=clipped,
                        value=val, table_seed=np.int64(INTERP_SEED))


def gen_interp_traj() -> None:
    sig = "power_grid_prop.signal_properties.mode"
    gen_traj("interp_sin_random", interp_overrides({sig: "sinusoidals", BPP + "interp_update_period": 40,
                                                    BPP + "interp_nb_agents": 20}),
             N=50, T=80, seed=8, controller="random", norm_ticks=(0, 80))
    gen_traj("interp_flat_dbbc_nosolar", interp_overrides({sig: "flat",
                                                           "cluster_prop.house_prop.solar_gain": False}),
             N=12, T=160, seed=3, controller="deadband_bbc", norm_ticks=(0,))


# ------------------------------------------------------------------------ services
def gen_services(N: int = 50, T: int = 120, seed: int = 4, start_stats_from: int = 30) -> None:
    """The reference's per-tick consumers along a ControllerManager-style loop
    (controller_manager.py:104-187: random.seed, three resets, then per tick update_data(obs) ->
    deadband bang-bang actions -> env.step -> Metrics.update(obs, next_obs, rewards, step)):
    Metrics' accumulators after every update (metrics_service.py:108-157) and the UI summary
    strings + graph data + house-list status counts (client_manager_service.py:62-245)."""
    import asyncio

    from app.services.client_manager_service import ClientManagerService, DESCRIPTION_KEYS
    from app.services.metrics_service import Metrics

    props = make_props({"cluster_prop.nb_agents": N, "power_grid_prop.signal_properties.mode": "sinusoidals"})
    random.seed(seed)
    env = Environment(props)
    obs = env.reset()
    obs = env.reset()
    met = Metrics(sys.modules["app.services.wandb_service"].WandbManager())
    met.initialize(N, start_stats_from, T)
    ui = ClientManagerService(None)
    ui.initialize_data(False)
    ctl = [DeadbandBangBangController({"id": i}, None) for i in range(N)]
    fields = ["cumul_avg_reward", "cumul_temp_offset", "cumul_temp_error", "cumul_signal_offset",
              "cumul_signal_error", "cumul_squared_error_temp", "max_temp_error", "cumul_OD_temp", "cumul_signal",
              "cumul_cons", "cumul_squared_error_sig", "cumul_squared_max_error_temp"]
    rec = {f: [] for f in fields}
    desc, graph, status = [], [], []
    for step in range(T):
        asyncio.run(ui.update_data(obs_dict=obs, time_step=step))
        desc.append([ui.description[step][k] for k in DESCRIPTION_KEYS])
        graph.append([ui.temp_diff[-1], ui.temp_err[-1], ui.air_temp[-1], ui.mass_temp[-1], ui.target_temp[-1],
                      ui.outdoor_temp[-1], ui.signal[-1], ui.consumption[-1]])
        hd = ui.houses_data[step]
        status.append([sum(h["hvacStatus"] == s for h in hd) for s in ("ON", "Lockout", "OFF")] +
                      [sum(h.get("secondsSinceOff", 0) for h in hd)])
        acts = {i: ctl[i].act(obs) for i in range(N)}
        nxt, rew = env.step(acts)
        met.update(obs, nxt, rew, step)
        for f in fields:
            rec[f].append(float(getattr(met, f)))
        obs = nxt
    met.update_rms(T)
    out = {f"metrics_{f}": np.array(v, np.float64) for f, v in rec.items()}
    out["rms"] = np.array([met.rmse_sig_per_ag, met.rmse_temp, met.rms_max_error_temp], np.float64)
    out["ui_graph"] = np.array(graph, np.float64)
    out["ui_status"] = np.array(status, np.int64)
    out["ui_desc_json"] = np.frombuffer(json.dumps(desc).encode(), np.uint8)
    meta = {"N": N, "T": T, "seed": seed, "start_stats_from": start_stats_from, "resets": 3,
            "controller": "deadband_bbc", "signal": "sinusoidals", "keys": list(DESCRIPTION_KEYS)}
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(OUT, "services.npz"), **out)


# ------------------------------------------------------------------------ MAPPO update (§8(f) 2)
def gen_mappo(num_state: int = 14, T: int = 40, batch_size: int = 16, epochs: int = 3) -> None:
    """One reference MAPPO.update (mappo.py:128-217) at N = 2 houses, where the reference's critic
    width (num_state + 1) matches its input (state ++ the other house's action).  num_state = 14 is
    the obs width of a 2-house cluster.  Inputs are synthetic transitions (float32-exact states),
    stored through MAPPO.store_transition; the minibatch order comes from torch.manual_seed(123)."""
    import torch
    from app.core.agents.trainables.mappo import MAPPO, MAPPOProperties

    cfg = MAPPOProperties(batch_size=batch_size, ppo_update_time=epochs)
    agent = MAPPO(cfg, num_state=num_state, num_action=2, seed=1)
    init = {f"init_actor_{k}": v.detach().numpy().copy() for k, v in agent.actor_net.state_dict().items()}
    init.update({f"init_critic_{k}": v.detach().numpy().copy() for k, v in agent.critic_net.state_dict().items()})
    rs = np.random.RandomState(5)
    states = rs.normal(0, 1, (T + 1, 2, num_state)).astype(np.float32)
    actions = rs.randint(0, 2, (T, 2)).astype(np.int64)
    probs = rs.uniform(0.3, 0.9, (T, 2)).astype(np.float32)
    rewards = -rs.uniform(0, 2, (T, 2))
    done = np.array([(t % 20) == 19 for t in range(T)])
    for t in range(T):
        agent.last_actions = {0: int(actions[t, 0]), 1: int(actions[t, 1])}
        agent.last_probs = {0: float(probs[t, 0]), 1: float(probs[t, 1])}
        agent.store_transition([states[t, 0].astype(np.float64), states[t, 1].astype(np.float64)],
                               [states[t + 1, 0].astype(np.float64), states[t + 1, 1].astype(np.float64)],
                               {0: float(rewards[t, 0]), 1: float(rewards[t, 1])}, bool(done[t]))
    reward = [tr.reward for tr in agent.buffer]
    dn = [tr.done for tr in agent.buffer]
    R, Gt = 0, []
    for i in reversed(range(len(reward))):  # the update's own return loop (mappo.py:135-140)
        if dn[i]:
            R = 0
        R = reward[i] + agent.gamma * R
        Gt.insert(0, R)
    torch.manual_seed(123)
    agent.update(T)
    out = dict(init)
    out.update({f"final_actor_{k}": v.detach().numpy().copy() for k, v in agent.actor_net.state_dict().items()})
    out.update({f"final_critic_{k}": v.detach().numpy().copy() for k, v in agent.critic_net.state_dict().items()})
    out.update(states=states, actions=actions, probs=probs, rewards=rewards, done=done, Gt=np.array(Gt))
    meta = {"num_state": num_state, "T": T, "batch_size": batch_size, "ppo_update_time": epochs, "seed": 1,
            "update_seed": 123, "training_steps": agent.training_step}
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(OUT, "mappo.npz"), **out)


def main() -> None:
    if len(sys.argv) > 1:  # only the named generators, e.g. `make_golden.py gen_interp gen_interp_traj`
        for name in sys.argv[1:]:
            globals()[name]()
        return
    with open(os.path.join(OUT, "marl_env_prop.json"), "w") as f:
        json.dump(env_prop_json(), f, indent=1, sort_keys=True)
    gen_lockout()
    gen_thermal()
    gen_solar()
    gen_signal()
    gen_rewards()
    sig = "power_grid_prop.signal_properties.mode"
    gen_traj("c1_sin_dbbc", {sig: "sinusoidals"}, N=50, T=200, seed=4, controller="deadband_bbc")
    gen_traj("c1_flat_random", {sig: "flat"}, N=50, T=200, seed=4, controller="random")
    gen_traj("fixed_steps_bbc", {sig: "regular_steps", "start_datetime_mode": "fixed",
                                 "cluster_prop.house_prop.deadband": 0.5},
             N=37, T=150, seed=123, controller="bbc", resets=1)
    gen_traj("n400_random_common", {sig: "sinusoidals",
                                    "reward_prop.penalty_props.mode": "common_L2"},
             N=400, T=40, seed=0, controller="random", norm_ticks=(0, 40))
    gen_traj("n64_mixture_2d", {sig: "flat", "reward_prop.penalty_props.mode": "mixture",
                                "reward_prop.penalty_props.alpha_common_max": 0.5,
                                "cluster_prop.agents_comm_prop.mode": "neighbours_2D",
                                "cluster_prop.agents_comm_prop.row_size": 8,
                                "cluster_prop.house_prop.solar_gain": False,
                                "time_step": 60},
             N=64, T=60, seed=5, controller="deadband_bbc", norm_ticks=(0, 60))
    gen_traj("n30_maxerr_groups_hvacmsg", {sig: "sinusoidals",
                                           "reward_prop.penalty_props.mode": "common_max_error",
                                           "cluster_prop.agents_comm_prop.mode": "closed_groups",
                                           "cluster_prop.agents_comm_prop.max_nb_agents_communication": 4,
                                           "cluster_prop.message_prop.thermal": True,
                                           "cluster_prop.message_prop.hvac": True,
                                           "state_prop.hvac": True, "state_prop.thermal": True,
                                           "state_prop.solar_gain": True},
             N=30, T=50, seed=9, controller="random", norm_ticks=(0, 1, 50))
    gen_greedy()
    gen_comm()
    gen_rng_order()
    gen_policy()
    gen_interp()
    gen_interp_traj()
    gen_services()
    gen_mappo()
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
