"""HIP path (libmdr_hip.so through mdr_amd.Environment) vs the reference goldens and the oracle.

Tolerances (BASELINE.json north_star): lockout counters, on/off masks and seconds-since-off
bit-exact; temperatures, cluster power and rewards within 1e-5 relative — asserted here much
tighter (1e-10) since the kernels keep the reference's fp64 operation order; float32 observation
vectors within 2 float32 ulps of the float64 reference values cast to float32.
"""
import os
import random

import numpy as np
import pytest

import golden_util as gu
from oracle import env_np as O

pytestmark = pytest.mark.gpu

TEMP_RTOL = 1e-10


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def make_env(props, seed, resets, **kw):
    from mdr_amd.environment import Environment

    rng = random.Random(seed)
    env = Environment(props, rng=rng, **kw)
    obs = None
    for _ in range(resets - 1):
        obs = env.reset()
    return env, rng, obs


@pytest.mark.parametrize("name", gu.TRAJ_NAMES)
def test_golden_trajectory_dict_api(torch_gpu, name):
    """Environment.reset/step (dict API) on the GPU reproduces the reference trajectory."""
    d, meta = gu.traj(name)
    props = gu.props_from_overrides(meta["overrides"])
    env, rng, obs = make_env(props, meta["seed"], meta["resets"])
    if obs is None:
        obs = env.get_obs()
    N, T = meta["N"], meta["T"]
    interp = meta["overrides"].get(gu.BPP + "mode") == "interpolation"
    assert obs[0]["cluster_hvac_power"] == float(d["init_P"])
    assert obs[0]["reg_signal"] == float(d["init_S"])
    np.testing.assert_array_equal([obs[i]["Ua"] for i in range(N)], d["pop_Ua"])
    np.testing.assert_array_equal([obs[i]["target_temp"] for i in range(N)], d["pop_target_temp"])
    hp = props.cluster_prop.house_prop
    for t in range(T):
        if meta["controller"] == "deadband_bbc":
            acts = {i: obs[i]["indoor_temp"] > obs[i]["target_temp"] + hp.deadband / 2 or
                    (not obs[i]["indoor_temp"] < obs[i]["target_temp"] - hp.deadband / 2 and obs[i]["turned_on"])
                    for i in range(N)}
            np.testing.assert_array_equal([bool(acts[i]) for i in range(N)], d["actions"][t].astype(bool))
        elif meta["controller"] == "bbc":
            acts = {i: obs[i]["indoor_temp"] > obs[i]["target_temp"] for i in range(N)}
            np.testing.assert_array_equal([bool(acts[i]) for i in range(N)], d["actions"][t].astype(bool))
        else:
            acts = {i: bool(d["actions"][t, i]) for i in range(N)}
        obs, rew = env.step(acts)
        on = np.array([obs[i]["turned_on"] for i in range(N)])
        lock = np.array([obs[i]["lockout"] for i in range(N)])
        sso = np.array([obs[i]["seconds_since_off"] for i in range(N)])
        np.testing.assert_array_equal(on, d["traj_on"][t].astype(bool), err_msg=f"on t={t}")
        np.testing.assert_array_equal(lock, d["traj_lock"][t].astype(bool), err_msg=f"lock t={t}")
        np.testing.assert_array_equal(sso, d["traj_sso"][t], err_msg=f"sso t={t}")
        Tn = np.array([obs[i]["indoor_temp"] for i in range(N)])
        Tmn = np.array([obs[i]["mass_temp"] for i in range(N)])
        np.testing.assert_allclose(Tn, d["traj_T"][t], rtol=TEMP_RTOL, atol=0, err_msg=f"T t={t}")
        np.testing.assert_allclose(Tmn, d["traj_Tm"][t], rtol=TEMP_RTOL, atol=0, err_msg=f"Tm t={t}")
        np.testing.assert_allclose([rew[i] for i in range(N)], d["traj_reward"][t], rtol=1e-9, atol=1e-12)
        assert obs[0]["cluster_hvac_power"] == float(d["traj_P"][t])
        if interp:  # base power from interpolated post-step temperatures (exp: ulp-level vs numpy)
            np.testing.assert_allclose(obs[0]["reg_signal"], float(d["traj_S"][t]), rtol=TEMP_RTOL, atol=0)
        else:
            assert obs[0]["reg_signal"] == float(d["traj_S"][t])
        assert obs[0]["OD_temp"] == float(d["traj_Tod"][t])
        assert obs[0]["solar_gain"] == float(d["traj_G"][t])
        m0 = np.array([obs[i]["message"][0]["current_temp_diff_to_target"] for i in range(N)])
        np.testing.assert_allclose(m0, d["traj_msg0_diff"][t], rtol=1e-9, atol=1e-9)
        np.testing.assert_array_equal([obs[i]["message"][0]["curr_consumption"] for i in range(N)],
                                      d["traj_msg0_curr"][t])


@pytest.mark.parametrize("name", gu.TRAJ_NAMES)
def test_golden_obs_vector(torch_gpu, name):
    """The device norm_state_dict vector (obs_tensor) matches the reference's at the goldens' ticks."""
    d, meta = gu.traj(name)
    props = gu.props_from_overrides(meta["overrides"])
    env, rng, _ = make_env(props, meta["seed"], meta["resets"])
    N = meta["N"]
    ticks = sorted(int(k[6:]) for k in d.keys() if k.startswith("norm_t"))

    def check(t):
        got = env.obs_tensor().cpu().numpy()
        ref = d[f"norm_t{t}"].astype(np.float32)
        np.testing.assert_array_max_ulp(got, ref, maxulp=2)

    if 0 in ticks:
        check(0)
    for t in range(max(ticks)):
        acts = torch_gpu.from_numpy(d["actions"][t]).to("cuda")
        env.step_tensor(acts)
        if t + 1 in ticks:
            check(t + 1)


def oracle_and_env(props, seed, **kw):
    from mdr_amd.environment import Environment

    env = Environment(props, rng=random.Random(seed), **kw)
    ora = O.OracleEnv(props, random.Random(seed))
    return env, ora


@pytest.mark.parametrize("n", [1, 2, 257, 4099])
def test_random_actions_vs_oracle(torch_gpu, n):
    """Edge sizes (1 house, ragged last block) against the oracle over 60 ticks."""
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env, ora = oracle_and_env(props, 31)
    rs = np.random.RandomState(n)
    for t in range(60):
        a = rs.randint(0, 2, n).astype(np.uint8)
        r = env.step_tensor(torch_gpu.from_numpy(a).to("cuda")).cpu().numpy()
        o, rr = ora.step(a.astype(bool))
        st = env.shard.host_state()
        np.testing.assert_array_equal(st["on"], o["on"])
        np.testing.assert_array_equal(st["lock"], o["lock"])
        np.testing.assert_array_equal(st["sso"], o["sso"])
        np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)
        np.testing.assert_allclose(st["Tm"], o["Tm"], rtol=TEMP_RTOL, atol=0)
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)
        assert env.cluster.current_power_consumption == o["P"]


@pytest.mark.parametrize("mode", ["common_L2", "common_max_error", "mixture"])
def test_common_penalty_modes_vs_oracle(torch_gpu, mode):
    props = gu.props_from_overrides({"cluster_prop.nb_agents": 3001,
                                     "power_grid_prop.signal_properties.mode": "flat",
                                     "reward_prop.penalty_props.mode": mode,
                                     "reward_prop.penalty_props.alpha_common_max": 0.5,
                                     "cluster_prop.house_prop.deadband": 0.4})
    env, ora = oracle_and_env(props, 5)
    rs = np.random.RandomState(2)
    for t in range(25):
        a = rs.randint(0, 2, 3001).astype(np.uint8)
        r = env.step_tensor(torch_gpu.from_numpy(a).to("cuda")).cpu().numpy()
        _, rr = ora.step(a.astype(bool))
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("ctrl", ["bangbang", "deadband_bangbang"])
def test_fused_bangbang_matches_dict_controller(torch_gpu, ctrl):
    """In-kernel controller (+ lookahead counts) == the reference controller applied per tick."""
    props = gu.props_from_overrides({"cluster_prop.nb_agents": 777,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals",
                                     "cluster_prop.house_prop.deadband": 0.5})
    env, ora = oracle_and_env(props, 8)
    hp = props.cluster_prop.house_prop
    for t in range(80):
        if ctrl == "bangbang":
            a = O.bangbang(ora.T, ora.pop["target"])
        else:
            a = O.deadband_bangbang(ora.T, ora.pop["target"], hp.deadband, ora.on)
        r = env.step_tensor(None, action_mode=ctrl, lookahead=ctrl).cpu().numpy()
        o, rr = ora.step(a)
        st = env.shard.host_state()
        np.testing.assert_array_equal(st["on"], o["on"])
        np.testing.assert_array_equal(st["lock"], o["lock"])
        np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)


def test_rollout_equals_steps(torch_gpu):
    """mdr_rollout (temporally blocked windows, exact thermal form) == the same ticks via step_tensor."""
    torch = torch_gpu
    props = gu.props_from_overrides({"cluster_prop.nb_agents": 20000,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    from mdr_amd.environment import Environment

    e1 = Environment(props, rng=random.Random(3), population="synthetic", seed=77)
    e2 = Environment(props, rng=random.Random(3), population="synthetic", seed=77)
    e1.shard.set_option("window_thermal", 0)  # MDR_THERMAL_EXACT: bit-identical to the one-tick kernels
    R = e1.rollout(50, action_mode="random")
    R2 = e1.rollout(50, action_mode="random")  # graph replay
    rews = []
    for t in range(100):
        rews.append(e2.step_tensor(None, action_mode="random").clone())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(torch.cat([R, R2]).cpu().numpy(), torch.stack(rews).cpu().numpy())
    s1, s2 = e1.shard.host_state(), e2.shard.host_state()
    for k in s1:
        np.testing.assert_array_equal(s1[k], s2[k])
    assert e1._cluster_power() == e2._cluster_power()  # rollout's p_out = last tick's P
    np.testing.assert_array_equal(e1.obs_tensor().cpu().numpy(), e2.obs_tensor().cpu().numpy())


def test_rollout_buffer_actions_vs_oracle(torch_gpu):
    torch = torch_gpu
    n, T = 3000, 40
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "flat"})
    env, ora = oracle_and_env(props, 12)
    acts = np.random.RandomState(0).randint(0, 2, (T, n)).astype(np.uint8)
    R = env.rollout(T, actions=torch.from_numpy(acts).cuda(), action_mode="buffer").cpu().numpy()
    for t in range(T):
        o, rr = ora.step(acts[t].astype(bool))
        np.testing.assert_allclose(R[t], rr, rtol=1e-9, atol=1e-12)
    st = env.shard.host_state()
    np.testing.assert_array_equal(st["sso"], o["sso"])
    np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)


def test_greedy_golden(torch_gpu):
    """mdr_ctrl_greedy on the reference's greedy inputs (F7) picks the reference's houses."""
    torch = torch_gpu
    from mdr_amd.environment import Environment

    d = gu.load("greedy.npz")
    Tn, N = d["action"].shape
    props = gu.props_from_overrides({"cluster_prop.nb_agents": N,
                                     "power_grid_prop.signal_properties.mode": "flat"})
    env = Environment(props, rng=random.Random(1))
    sh = env.shard
    from mdr_amd.shard import encode_hvac

    for t in range(Tn):
        caps = [int(c) for c in d["cap"][t]]
        idx = np.array([env._cap_values.index(c) for c in caps], np.uint8)
        sh.cap_idx.copy_(torch.from_numpy(idx).cuda())
        sh.t_air.copy_(torch.from_numpy(d["T"][t]).cuda())
        sh.target.copy_(torch.from_numpy(d["target"][t]).cuda())
        sh.hvac.copy_(torch.from_numpy(encode_hvac(np.ones(N, bool), d["lock"][t], np.zeros(N))).cuda())
        out = torch.zeros(N, dtype=torch.uint8, device="cuda")
        sh.greedy(float(d["S"][t]), out)
        np.testing.assert_array_equal(out.cpu().numpy().astype(bool), d["action"][t].astype(bool), err_msg=f"t={t}")


def test_greedy_vs_oracle_large(torch_gpu):
    torch = torch_gpu
    from mdr_amd.environment import Environment

    n = 200_000
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "flat"})
    env = Environment(props, rng=random.Random(1), population="synthetic", seed=5)
    for t in range(5):
        env.step_tensor(None, action_mode="random")
    sh = env.shard
    st, prm = sh.host_state(), sh.host_params()
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    for S in (0.0, 3000.0, 1.0e8, float(env.power_grid.current_signal), 1e12):
        out = torch.zeros(n, dtype=torch.uint8, device="cuda")
        sh.greedy(S, out)
        ref = O.greedy(st["T"], prm["target"], caps, props.cluster_prop.house_prop.hvac_prop.cop, st["lock"], S)
        np.testing.assert_array_equal(out.cpu().numpy().astype(bool), ref)


@pytest.mark.parametrize("form", ["select", "sort"])
def test_greedy_key_runs_vs_oracle(torch_gpu, form):
    """mdr_ctrl_greedy on adversarial key layouts, in both forms (select: the default histogram
    select; sort: MDR_OPT_GREEDY_SORT, the full 64-bit key sort): 300 identical temperatures, 700 keys
    1e-9 apart in DESCENDING house order, 100 houses at exactly their target (key -0.0), random
    lockouts, budgets that put the pivot inside each group; the oracle's stable numpy order
    decides.  The select form's window decides all of these; a cluster of identical keys (one bin
    of every house) goes to its exact in-kernel fallback and still matches."""
    torch = torch_gpu
    from mdr_amd.environment import Environment
    from mdr_amd.shard import encode_hvac

    n = 50_000
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "flat"})
    env = Environment(props, rng=random.Random(3), population="synthetic", seed=8)
    sh = env.shard
    sh.set_option("greedy_sort", form == "sort")
    prm = sh.host_params()
    rs = np.random.RandomState(5)
    tg = prm["target"].copy()
    T = tg + rs.normal(0.0, 1.5, n)
    T[1000:1300] = 23.25                                  # identical keys (per house target differs: set it)
    tg[1000:1300] = 22.0
    T[2000:2700] = 22.5 + 1e-9 * np.arange(700)           # keys -(0.5 + i 1e-9): descending in house order
    tg[2000:2700] = 22.0
    T[3000:3100] = tg[3000:3100]                          # key -0.0
    lock = rs.rand(n) < 0.3
    sh.t_air.copy_(torch.from_numpy(T).cuda())
    sh.target.copy_(torch.from_numpy(tg).cuda())
    sh.hvac.copy_(torch.from_numpy(encode_hvac(np.zeros(n, bool), lock, np.full(n, 5))).cuda())
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    cop = props.cluster_prop.house_prop.hvac_prop.cop
    key = -(T - tg)
    order = np.argsort(key, kind="stable")
    pw = caps[order] / cop
    cum = np.cumsum(pw)
    budgets = [0.0, 1e12, float(cum[n // 2])]
    for grp in (slice(1000, 1300), slice(2000, 2700), slice(3000, 3100)):  # pivot inside each group
        pos = np.nonzero(np.isin(order, np.arange(n)[grp]))[0]
        budgets += [float(cum[pos[len(pos) // 2]] - 1.0), float(cum[pos[len(pos) // 2]] + 0.5)]
    f0 = sh.greedy_fallbacks()
    for S in budgets:
        out = torch.zeros(n, dtype=torch.uint8, device="cuda")
        sh.greedy(S, out)
        ref = O.greedy(T, tg, caps, cop, lock, S)
        np.testing.assert_array_equal(out.cpu().numpy().astype(bool), ref, err_msg=f"S={S}")
    assert sh.greedy_fallbacks() == f0  # (the window decided every one of these)
    # every key identical: one bin of n houses > the window -> the sort form decides
    sh.t_air.copy_(torch.full((n,), 23.0, dtype=torch.float64, device="cuda"))
    sh.target.copy_(torch.full((n,), 22.0, dtype=torch.float64, device="cuda"))
    for S in (float(cum[n // 3]), 1e12):
        out = torch.zeros(n, dtype=torch.uint8, device="cuda")
        sh.greedy(S, out)
        ref = O.greedy(np.full(n, 23.0), np.full(n, 22.0), caps, cop, lock, S)
        np.testing.assert_array_equal(out.cpu().numpy().astype(bool), ref, err_msg=f"equal keys S={S}")
    if form == "select":
        # the n identical keys make one bin of n houses > the window: decided by k_gq_select's exact
        # in-kernel fallback (S = 1e12 takes everything: decided by the superbins)
        assert sh.greedy_fallbacks() == f0 + 1


@pytest.mark.parametrize("n", [3001, 200_003])
def test_greedy_keys_with_lookahead_keeps_counts(torch_gpu, n):
    """a step with a lookahead AND ctrl='greedy_keys' must keep the lookahead's counts
    (k_gq_keys used to zero that slab, so the next non-greedy step ran with P = 0), and a greedy call
    after such a step must still count only its own decisions.  Twins: the same seeds with and
    without the keys; everything compared with ==."""
    torch = torch_gpu
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    a = Environment(props, rng=random.Random(5), population="synthetic", seed=5)
    b = Environment(props, rng=random.Random(5), population="synthetic", seed=5)
    for _ in range(3):
        ra = a.step_tensor(None, action_mode="random", lookahead="random", ctrl="greedy_keys").clone()
        rb = b.step_tensor(None, action_mode="random", lookahead="random").clone()
        assert torch.equal(ra, rb)
    ra = a.step_tensor(None, action_mode="random").clone()  # (the counts the keys' step looked ahead)
    rb = b.step_tensor(None, action_mode="random").clone()
    assert torch.equal(ra, rb)
    assert a.cluster.current_power_consumption == b.cluster.current_power_consumption > 0
    sa, sb = a.shard.host_state(), b.shard.host_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    # keys + lookahead, then the greedy decision and its step: the decisions' counts alone
    a.step_tensor(None, action_mode="random", lookahead="random", ctrl="greedy_keys")
    b.step_tensor(None, action_mode="random", lookahead="random")
    ga, gb = a.greedy_actions(), b.greedy_actions()
    assert torch.equal(ga, gb)
    ra, rb = a.step_tensor(ga).clone(), b.step_tensor(gb).clone()
    assert torch.equal(ra, rb)
    prm = a.shard.host_params()
    caps = np.array(a._cap_values, np.float64)[prm["cap_idx"]]
    on = a.shard.host_state()["on"]
    P = float(np.sum(np.where(on, caps / props.cluster_prop.house_prop.hvac_prop.cop, 0.0)))
    assert a.cluster.current_power_consumption == b.cluster.current_power_consumption == P


def test_one_million_houses_properties(torch_gpu):
    """Full-size (1,048,576 houses) size-independent checks: FSM bit-exact vs the oracle on the
    same input state, temperatures within tolerance, P == sum of ON power (exact integers)."""
    torch = torch_gpu
    from mdr_amd.environment import Environment

    n = 1 << 20
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(9), population="synthetic", seed=9)
    for _ in range(30):
        env.step_tensor(None, action_mode="random", lookahead="random")
    sh = env.shard
    st0, prm = sh.host_state(), sh.host_params()
    a = (torch.rand(n, device="cuda") < 0.5).to(torch.uint8)
    tick_tod, tick_S = env.current_od_temp, env.power_grid.current_signal
    r = env.step_tensor(a).cpu().numpy()
    st1 = sh.host_state()
    hv = props.cluster_prop.house_prop.hvac_prop
    on, lock, sso = O.hvac_step(st0["on"], st0["lock"], st0["sso"], a.cpu().numpy().astype(bool),
                                hv.lockout_duration, props.time_step.seconds)
    np.testing.assert_array_equal(st1["on"], on)
    np.testing.assert_array_equal(st1["lock"], lock)
    np.testing.assert_array_equal(st1["sso"], sso)
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    q = O.heat_transfer(on, caps, hv.latent_cooling_fraction)
    T, Tm = O.update_temperature(st0["T"], st0["Tm"], prm["ua"], prm["ca"], prm["cm"], prm["hm"], q,
                                 env._solar, tick_tod, float(props.time_step.seconds))
    np.testing.assert_allclose(st1["T"], T, rtol=TEMP_RTOL, atol=0)
    np.testing.assert_allclose(st1["Tm"], Tm, rtol=TEMP_RTOL, atol=0)
    P = float(np.sum(np.where(on, caps / hv.cop, 0.0)))
    assert env.cluster.current_power_consumption == P
    rr = O.rewards(T, prm["target"], props.cluster_prop.house_prop.deadband, P, tick_S,
                   props.reward_prop, props.cluster_prop.house_prop.target_temp)
    np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)
    assert np.all(np.isfinite(r))


def test_greedy_one_million_vs_oracle(torch_gpu):
    """Config C3 at its stated size: 1,048,576 houses, device GreedyMyopic on the post-step state
    -> env.step, 4 ticks, against the oracle's greedy (stable order) and step on the same population:
    actions and on/lock/sso exact, temperatures rtol 1e-10, rewards, P."""
    from mdr_amd.environment import Environment

    n = 1 << 20
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(21), population="synthetic", seed=21)
    prm = env.shard.host_params()
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    pop = {"Ua": prm["ua"], "Ca": prm["ca"], "Cm": prm["cm"], "Hm": prm["hm"], "target": prm["target"], "cap": caps}
    ora = O.OracleEnv(props, random.Random(21), population=pop)
    hv = props.cluster_prop.house_prop.hvac_prop
    for t in range(4):
        assert float(env.power_grid.current_signal) == float(ora.S)
        a = env.greedy_actions().cpu().numpy().astype(bool)
        ref = O.greedy(ora.T, ora.pop["target"], caps, hv.cop, ora.lock, float(ora.S))
        np.testing.assert_array_equal(a, ref, err_msg=f"greedy t={t}")
        r = env.step_tensor(torch_gpu.from_numpy(a.astype(np.uint8)).to("cuda")).cpu().numpy()
        o, rr = ora.step(a)
        st = env.shard.host_state()
        np.testing.assert_array_equal(st["on"], o["on"])
        np.testing.assert_array_equal(st["lock"], o["lock"])
        np.testing.assert_array_equal(st["sso"], o["sso"])
        np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)
        assert env.cluster.current_power_consumption == o["P"]


def test_greedy_four_million_vs_oracle(torch_gpu):
    """4,194,304 houses: k_gq_compact runs 1,024 blocks of 1,024 threads, more than the chip holds
    at once, so later blocks start after block 0 has published the window (r03's race: block 0
    overwrote the crossing base those blocks still read, and they cut a different window).  The
    device greedy + step == the oracle's over 3 ticks, every call decided by the window (no exact
    fallback); the steps write the next call's keys (ctrl='greedy_keys'), so calls 2 and 3 may cut
    their window from the predicted band in k_gq_binsc's 1,024 blocks."""
    from mdr_amd.environment import Environment

    n = 1 << 22
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(23), population="synthetic", seed=23)
    prm = env.shard.host_params()
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    pop = {"Ua": prm["ua"], "Ca": prm["ca"], "Cm": prm["cm"], "Hm": prm["hm"], "target": prm["target"], "cap": caps}
    ora = O.OracleEnv(props, random.Random(23), population=pop)
    hv = props.cluster_prop.house_prop.hvac_prop
    for t in range(3):
        a = env.greedy_actions().cpu().numpy().astype(bool)
        ref = O.greedy(ora.T, ora.pop["target"], caps, hv.cop, ora.lock, float(ora.S))
        np.testing.assert_array_equal(a, ref, err_msg=f"greedy t={t}")
        r = env.step_tensor(torch_gpu.from_numpy(a.astype(np.uint8)).to("cuda"), ctrl="greedy_keys").cpu().numpy()
        o, rr = ora.step(a)
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)
        assert env.cluster.current_power_consumption == o["P"]
    st = env.shard.host_state()
    for k in ("on", "lock", "sso"):
        np.testing.assert_array_equal(st[k], o[k], err_msg=k)
    d = env.shard.greedy_state()
    assert d["calls"] == 3 and d["fallbacks"] == 0, d
    print("band", env.shard.greedy_band())


@pytest.mark.parametrize("path", ["step", "rollout"])
def test_perlin_trajectory_vs_oracle(torch_gpu, path):
    """Perlin signal mode (the MARLconfig default) on the GPU path, against the
    oracle fed an independent scalar restatement of the same published algorithm
    (oracle/perlin_np.py; parity with the absent third-party package is UNPINNED).  The seed is
    drawn in the reference's order (signal_calculator.py:24-31).  'step': dict-free step_tensor
    ticks with buffer actions; 'rollout': the default rollout (direct launches, perlin tabulated per
    date into the C host drivers, affine windows) with the replayed Philox actions, crossing
    midnight.  Signal within 1e-12 relative (the two restatements round the fade's powers
    differently), masks exact, temperatures rtol 1e-10, rewards rtol 1e-9."""
    import datetime as dt

    import philox_np as PX

    torch = torch_gpu
    from mdr_amd.environment import Environment

    n, T = 4099, 240
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "perlin"})
    props.start_datetime = dt.datetime(2021, 6, 30, 23, 50)
    props.start_datetime_mode = "fixed"
    env = Environment(props, rng=random.Random(17), seed=99)
    ora = O.OracleEnv(props, random.Random(17))
    np.testing.assert_allclose(float(env.power_grid.current_signal), ora.S, rtol=1e-12)
    assert env._vector_drivers_ok()
    gids = np.arange(n, dtype=np.uint64)
    if path == "rollout":
        tick0 = env._tick
        R = env.rollout(T, action_mode="random").cpu().numpy()
        for t in range(T):
            o, rr = ora.step(PX.random_actions(99, gids, tick0 + t))
            np.testing.assert_allclose(R[t], rr, rtol=1e-9, atol=1e-12, err_msg=f"reward t={t}")
    else:
        rs = np.random.RandomState(3)
        for t in range(T):
            a = rs.randint(0, 2, n).astype(np.uint8)
            r = env.step_tensor(torch.from_numpy(a).to("cuda")).cpu().numpy()
            o, rr = ora.step(a.astype(bool))
            np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12, err_msg=f"reward t={t}")
            np.testing.assert_allclose(float(env.power_grid.current_signal), o["S"], rtol=1e-12)
    st = env.shard.host_state()
    for k in ("on", "lock", "sso"):
        np.testing.assert_array_equal(st[k], o[k], err_msg=k)
    np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)
    np.testing.assert_allclose(float(env.power_grid.current_signal), o["S"], rtol=1e-12)
    assert env.cluster.current_power_consumption == o["P"]
    assert env.date_time == o["date"] and env.date_time.day == 1  # crossed midnight into July



def _greedy_env(n, seed, signal="sinusoidals"):
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": signal})
    return props, Environment(props, rng=random.Random(seed), population="synthetic", seed=seed)


def test_greedy_loop_keys_epilogue_and_counts(torch_gpu):
    """Config C3's loop as the bench runs it: greedy_actions (its launches also count the ON houses
    of the decided actions) -> step_tensor(ctrl='greedy_keys') (one launch: those counts, and the
    next greedy call's keys written by the step kernel's epilogue) == the same decisions through a
    twin that recomputes keys (k_gq_keys) and counts (mdr_power_counts) every tick, and == the
    oracle's greedy + step; 12 ticks at 200,003 houses (ragged tiles)."""
    torch = torch_gpu
    n = 200_003
    props, a = _greedy_env(n, 23)
    _, b = _greedy_env(n, 23)
    prm = a.shard.host_params()
    caps = np.array(a._cap_values, np.float64)[prm["cap_idx"]]
    pop = {"Ua": prm["ua"], "Ca": prm["ca"], "Cm": prm["cm"], "Hm": prm["hm"], "target": prm["target"], "cap": caps}
    ora = O.OracleEnv(props, random.Random(23), population=pop)
    cop = props.cluster_prop.house_prop.hvac_prop.cop
    ga = torch.empty(n, dtype=torch.uint8, device="cuda")
    for t in range(12):
        aa = a.greedy_actions(out=ga)
        ab = b.greedy_actions().clone()  # another buffer: its step recounts with mdr_power_counts
        assert torch.equal(aa, ab), t
        ref = O.greedy(ora.T, ora.pop["target"], caps, cop, ora.lock, float(ora.S))
        np.testing.assert_array_equal(aa.cpu().numpy().astype(bool), ref, err_msg=f"greedy t={t}")
        ra = a.step_tensor(aa, ctrl="greedy_keys").clone()
        rb = b.step_tensor(ab).clone()
        assert torch.equal(ra, rb), t
        o, rr = ora.step(ref)
        np.testing.assert_allclose(ra.cpu().numpy(), rr, rtol=1e-9, atol=1e-12)
        assert a.cluster.current_power_consumption == o["P"]
    st = a.shard.host_state()
    np.testing.assert_array_equal(st["on"], o["on"])
    np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)
    bd = a.shard.greedy_band()
    assert bd["calls"] == 12 and bd["skips"] >= 1, bd  # (the twin never skips: its keys are k_gq_keys')
    assert b.shard.greedy_band()["skips"] == 0


@pytest.mark.parametrize("strided", [False, True])
def test_greedy_rollout_matches_loop(torch_gpu, strided):
    """Environment.greedy_rollout (mdr_greedy_rollout: config C3's loop in one C call, drivers from
    driver_window) == the per-tick Python loop greedy_actions -> step_tensor(ctrl='greedy_keys') on a
    twin: every tick's actions and rewards bit for bit, the state, clock and signal after; 13 ticks
    at 200,003 houses (ragged tiles), per-tick buffers ('strided') or one overwritten buffer."""
    torch = torch_gpu
    n, T = 200_003, 13
    _, a = _greedy_env(n, 29)
    _, b = _greedy_env(n, 29)
    if strided:
        acts, rews = a.greedy_rollout(T, actions=torch.empty((T, n), dtype=torch.uint8, device="cuda"))
    else:
        acts, rews = a.greedy_rollout(T, rewards=torch.empty(n, dtype=torch.float64, device="cuda"))
    ga = torch.empty(n, dtype=torch.uint8, device="cuda")
    for t in range(T):
        ab = b.greedy_actions(out=ga)
        rb = b.step_tensor(ab, ctrl="greedy_keys")
        if strided:
            assert torch.equal(acts[t], ab), t
            assert torch.equal(rews[t], rb), t
    if not strided:
        assert torch.equal(acts, ab) and torch.equal(rews, rb)
    sa, sb = a.shard.host_state(), b.shard.host_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    assert a.date_time == b.date_time and a._tick == b._tick
    assert float(a.power_grid.current_signal) == float(b.power_grid.current_signal)
    assert float(a.current_od_temp) == float(b.current_od_temp)
    assert a.cluster.current_power_consumption == b.cluster.current_power_consumption


@pytest.mark.parametrize("n,signal,T", [(17, "sinusoidals", 10), (4097, "regular_steps", 20),
                                        (3001, "sinusoidals", 30), (200_003, "sinusoidals", 40),
                                        (1 << 20, "sinusoidals", 40), (1 << 20, "regular_steps", 40),
                                        (1 << 20, "perlin", 40), (1 << 22, "sinusoidals", 12)])
def test_greedy_fused_matches_per_tick(torch_gpu, n, signal, T):
    """The fused tick (MDR_OPT_GQ_FUSED: k_gq_decide2 -> k_step_pipe<..., GQ = 2>, the decision applied
    from the pre-step keys) against the per-tick form (mdr_ctrl_greedy + mdr_step, itself pinned to
    the oracle and to the Python loop) on twins: every tick's actions and rewards bit for bit, the
    state after, for the sinusoidal, regular-steps (a budget jump at every step edge) and perlin
    signals, ragged and 4M-house clusters; the fused counters (band hits, misses, exact) printed."""
    torch = torch_gpu
    _, a = _greedy_env(n, 53, signal)
    _, b = _greedy_env(n, 53, signal)
    a.shard.set_option("gq_fused", 1)
    b.shard.set_option("gq_fused", 0)
    acts_a = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    acts_b = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    ra = a.greedy_rollout(T, actions=acts_a)[1]
    rb = b.greedy_rollout(T, actions=acts_b)[1]
    for t in range(T):
        assert torch.equal(acts_a[t], acts_b[t]), t
        assert torch.equal(ra[t], rb[t]), t
    sa, sb = a.shard.host_state(), b.shard.host_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    assert a.cluster.current_power_consumption == b.cluster.current_power_consumption
    fd = a.shard.greedy_fused_diag()
    print(signal, n, "fused", fd)
    assert fd["calls"] == T


@pytest.mark.parametrize("n", [200_003, 1 << 20])
def test_greedy_fused_jumping_budgets(torch_gpu, n):
    """The fused tick's miss path (the decision's own pass over the cluster, its last block sorting the
    window) and its hit path after it: mdr_greedy_rollout over 32 ticks whose budgets jump at random
    across the cluster's cumulative power every 4th tick and stay put in between, against the per-tick
    form on a twin fed the same ticks; actions, rewards, state bit for bit."""
    torch = torch_gpu
    from mdr_amd.environment import TickWindow

    props, a = _greedy_env(n, 59)
    _, b = _greedy_env(n, 59)
    a.shard.set_option("gq_fused", 1)
    b.shard.set_option("gq_fused", 0)
    T = 32
    ta = a.driver_window(T)
    tb = TickWindow(ta.a.copy())
    b.driver_window(T)  # (the twin's clock, unused)
    prm = a.shard.host_params()
    p_all = float(np.sum(np.array(a._cap_values, np.float64)[prm["cap_idx"]]) /
                  props.cluster_prop.house_prop.hvac_prop.cop)
    rs = np.random.RandomState(11)
    S = p_all * np.repeat(rs.uniform(0.05, 0.95, T // 4), 4)
    ta.s_prev[:] = S
    tb.s_prev[:] = S
    out = []
    for e, tw in ((a, ta), (b, tb)):
        acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
        rews = torch.empty((T, n), dtype=torch.float64, device="cuda")
        e.shard.greedy_rollout(tw, acts, n, rews, n)
        out.append((acts, rews, e.shard.host_state()))
    for t in range(T):
        assert torch.equal(out[0][0][t], out[1][0][t]), t
        assert torch.equal(out[0][1][t], out[1][1][t]), t
    for k in out[0][2]:
        np.testing.assert_array_equal(out[0][2][k], out[1][2][k], err_msg=k)
    fd = a.shard.greedy_fused_diag()
    print("jumping budgets", n, fd)
    assert fd["calls"] == T and fd["misses"] + fd["exact"] >= 1


@pytest.mark.parametrize("case", ["nan_crossing", "identical_crossing", "after_state_write"])
def test_greedy_fused_exact_and_restart(torch_gpu, case):
    """The fused tick where the window cannot decide (a crossing among NaN keys, 10,000 identical keys
    around the crossing: gq_exact, kGqfFull) and after the state was rewritten between two rollouts
    (the producer k_gq_keys2 runs again): == the per-tick form on a twin, 4 ticks."""
    torch = torch_gpu
    from mdr_amd.shard import encode_hvac

    n = 60_000
    envs = [_greedy_env(n, 31)[1], _greedy_env(n, 31)[1]]
    envs[0].shard.set_option("gq_fused", 1)
    envs[1].shard.set_option("gq_fused", 0)
    outs = []
    for e in envs:
        sh = e.shard
        prm = sh.host_params()
        rs = np.random.RandomState(7)
        tg = prm["target"].copy()
        T = tg + rs.normal(0.0, 1.0, n)
        lock = rs.rand(n) < 0.3
        if case == "nan_crossing":
            T[rs.choice(n, 40000, replace=False)] = np.nan
        elif case == "identical_crossing":
            T[:50000] = 24.0
            tg[:50000] = 22.5
        if case == "after_state_write":
            e.greedy_rollout(3)
        sh.t_air.copy_(torch.from_numpy(T).cuda())
        sh.target.copy_(torch.from_numpy(tg).cuda())
        sh.hvac.copy_(torch.from_numpy(encode_hvac(~lock & (rs.rand(n) < 0.5), lock, rs.randint(0, 60, n))).cuda())
        sh.params_changed()
        acts = torch.empty((4, n), dtype=torch.uint8, device="cuda")
        r = e.greedy_rollout(4, actions=acts)[1]
        outs.append((acts.clone(), r.clone(), sh.host_state()))
    (aa, ra, sa), (ab, rb, sb) = outs
    assert torch.equal(aa, ab)
    assert torch.equal(ra, rb)
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    print(case, envs[0].shard.greedy_fused_diag())


@pytest.mark.parametrize("n", [200_003, 1 << 20])
def test_greedy_band_forms_agree(torch_gpu, n):
    """The band's two launches (k_gq_binsc + k_gq_finish) against the r04 three (MDR_OPT_GQ_BAND 0)
    on twin environments: 24 ticks of C3's loop (mostly band hits), then 12 calls at budgets drawn
    at random across the cluster's cumulative power (mostly misses: k_gq_finish cuts the window,
    compacts and ranks it in its last block), each followed by a GQ step; actions and rewards bit
    for bit, the same state after."""
    torch = torch_gpu
    props, a = _greedy_env(n, 37)
    _, b = _greedy_env(n, 37)
    b.shard.set_option("gq_band", 0)
    for e in (a, b):  # (the per-tick forms: mdr_ctrl_greedy + mdr_step, not the fused tick)
        e.shard.set_option("gq_fused", 0)
    ra, rb = a.greedy_rollout(24)[1], b.greedy_rollout(24)[1]
    assert torch.equal(ra, rb)
    prm = a.shard.host_params()
    p_all = float(np.sum(np.array(a._cap_values, np.float64)[prm["cap_idx"]]) /
                  props.cluster_prop.house_prop.hvac_prop.cop)
    rs = np.random.RandomState(5)
    ga = torch.empty(n, dtype=torch.uint8, device="cuda")
    gb = torch.empty(n, dtype=torch.uint8, device="cuda")
    for t in range(12):
        S = p_all * float(rs.uniform(0.02, 0.98))
        a.shard.greedy(S, ga)
        b.shard.greedy(S, gb)
        assert torch.equal(ga, gb), t
        r1 = a.step_tensor(ga, ctrl="greedy_keys")
        r2 = b.step_tensor(gb, ctrl="greedy_keys")
        assert torch.equal(r1, r2), t
    sa, sb = a.shard.host_state(), b.shard.host_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    print("band", a.shard.greedy_band())


def test_greedy_band_skips_and_misses(torch_gpu):
    """The predicted band (k_gq_binsc): config C3's loop at 1,048,576 houses, 16 ticks, against the
    oracle's greedy + step every tick, through every way a call meets the band: predicted ticks
    (the window cut from the step epilogue's band, no bins pass), a forced miss (tick 6 decides a
    budget at 10% of the cluster's cumulative power, far outside the band: the bins pass runs), the
    tick after it (the band re-centred on the miss), and two GQ steps with no greedy call between
    (tick 11: the first step's histograms are zeroed before the second's epilogue adds its own)."""
    torch = torch_gpu
    n = 1 << 20
    props, env = _greedy_env(n, 41)
    sh = env.shard
    prm = sh.host_params()
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    pop = {"Ua": prm["ua"], "Ca": prm["ca"], "Cm": prm["cm"], "Hm": prm["hm"], "target": prm["target"], "cap": caps}
    ora = O.OracleEnv(props, random.Random(41), population=pop)
    cop = props.cluster_prop.house_prop.hvac_prop.cop
    ga = torch.empty(n, dtype=torch.uint8, device="cuda")
    log = []
    for t in range(16):
        before = sh.greedy_band()["skips"] if t in (6, 7) else None
        if t == 6:
            key = -(ora.T - ora.pop["target"])
            order = np.argsort(key, kind="stable")
            S = float(np.cumsum((caps / cop)[order])[n // 10]) + 0.25
            sh.greedy(S, ga)
            aa = ga
        else:
            S = float(ora.S)
            aa = env.greedy_actions(out=ga)
        ref = O.greedy(ora.T, ora.pop["target"], caps, cop, ora.lock, S)
        np.testing.assert_array_equal(aa.cpu().numpy().astype(bool), ref, err_msg=f"greedy t={t}")
        if t == 6:
            assert sh.greedy_band()["skips"] == before, "a budget outside the band must run the bins pass"
        r = env.step_tensor(aa, ctrl="greedy_keys").cpu().numpy()
        o, rr = ora.step(ref)
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12, err_msg=f"reward t={t}")
        assert env.cluster.current_power_consumption == o["P"], t
        if t == 11:  # a second GQ step before the next greedy call
            z = torch.zeros(n, dtype=torch.uint8, device="cuda")
            r = env.step_tensor(z, ctrl="greedy_keys").cpu().numpy()
            o, rr = ora.step(np.zeros(n, bool))
            np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)
        log.append(sh.greedy_band())
    st = sh.host_state()
    for k in ("on", "lock", "sso"):
        np.testing.assert_array_equal(st[k], o[k], err_msg=k)
    np.testing.assert_allclose(st["T"], o["T"], rtol=TEMP_RTOL, atol=0)
    bd = sh.greedy_band()
    print("band", bd, [d["band_base"] for d in log])
    assert bd["calls"] == 16, bd
    assert bd["skips"] >= 8, (bd, log)  # (ticks 0, 6 and 7 cannot skip; 12 may not)


@pytest.mark.parametrize("case", ["nan_crossing", "nan_after", "identical_crossing"])
def test_greedy_exact_fallback(torch_gpu, case):
    """Inputs the candidate window cannot decide go to k_gq_select's exact in-kernel radix select
    (no host synchronisation): a crossing among NaN keys (NaN temperatures sort last, in house order,
    as numpy's stable argsort and pandas' na_position='last' put them), NaN keys after the crossing,
    10,000 identical keys around the crossing; actions and the counted cluster power == the oracle."""
    torch = torch_gpu
    n = 60_000
    props, env = _greedy_env(n, 31)
    sh = env.shard
    prm = sh.host_params()
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    cop = props.cluster_prop.house_prop.hvac_prop.cop
    rs = np.random.RandomState(7)
    tg = prm["target"].copy()
    T = tg + rs.normal(0.0, 1.0, n)
    lock = rs.rand(n) < 0.3
    if case.startswith("nan"):
        T[rs.choice(n, 5000, replace=False)] = np.nan
    else:
        T[20000:30000] = 24.0
        tg[20000:30000] = 22.5
    sh.t_air.copy_(torch.from_numpy(T).cuda())
    sh.target.copy_(torch.from_numpy(tg).cuda())
    from mdr_amd.shard import encode_hvac

    sh.hvac.copy_(torch.from_numpy(encode_hvac(~lock & (rs.rand(n) < 0.5), lock, rs.randint(0, 60, n))).cuda())
    sh.params_changed()
    key = -(T - tg)
    order = np.argsort(key, kind="stable")
    cum = np.cumsum((caps / cop)[order])
    finite = int(np.isfinite(key).sum())
    if case == "nan_crossing":
        S = float(cum[finite + 1234]) - 0.5
    elif case == "nan_after":
        S = float(cum[finite // 2]) + 0.5
    else:
        pos = np.nonzero((order >= 20000) & (order < 30000))[0]
        S = float(cum[pos[len(pos) // 2]]) - 1.0
    f0 = sh.greedy_fallbacks()
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    sh.greedy(S, out)
    ref = O.greedy(T, tg, caps, cop, lock, S)
    np.testing.assert_array_equal(out.cpu().numpy().astype(bool), ref)
    if case != "nan_after":
        assert sh.greedy_fallbacks() >= f0 + 1
    # the counts the greedy launches left == the ON houses those actions produce
    st0 = sh.host_state()
    hv = props.cluster_prop.house_prop.hvac_prop
    on, _, _ = O.hvac_step(st0["on"], st0["lock"], st0["sso"], ref, hv.lockout_duration, props.time_step.seconds)
    env._counts_ready = ("greedy", out.data_ptr())
    env.step_tensor(out)
    assert env.cluster.current_power_consumption == float(np.sum(np.where(on, caps / cop, 0.0)))


@pytest.mark.parametrize("form", ["band", "fused"])
def test_greedy_state_write_remaps_keys(torch_gpu, form):
    """A state write that moves every key far outside the key map the last calls built (here 9 K
    warmer than target: keys near -9 against a map fitted around 0): the first call after it rebuilds
    the cells over the new key range (k_gq_remap) instead of clamping the cluster into the map's end
    cells, whose crossing bin would overflow the window and send the decision to gq_exact (one block
    over the cluster, ~7 ms at 1M houses).  No exact fallback on that call, and the decisions equal the
    sort form's (hipCUB radix sort + the reference's sequential rule) on a twin, actions and rewards
    bit for bit."""
    torch = torch_gpu
    from mdr_amd.shard import encode_hvac

    n = 300_017
    _, a = _greedy_env(n, 71)
    _, b = _greedy_env(n, 71)
    a.shard.set_option("gq_fused", 1 if form == "fused" else 0)
    b.shard.set_option("greedy_sort", 1)
    outs = []
    for e in (a, b):
        e.greedy_rollout(10)
        sh = e.shard
        prm = sh.host_params()
        rs = np.random.RandomState(13)
        tg = prm["target"].copy()
        T = tg + 9.0 + rs.normal(0.0, 1.0, n)
        lock = rs.rand(n) < 0.3
        sh.t_air.copy_(torch.from_numpy(T).cuda())
        sh.hvac.copy_(torch.from_numpy(encode_hvac(~lock & (rs.rand(n) < 0.5), lock, rs.randint(0, 60, n))).cuda())
        sh.params_changed()
        d0 = (sh.greedy_diag()["fallbacks"], sh.greedy_fused_diag()["exact"])
        acts = torch.empty((3, n), dtype=torch.uint8, device="cuda")
        r = e.greedy_rollout(3, actions=acts)[1]
        d1 = (sh.greedy_diag()["fallbacks"], sh.greedy_fused_diag()["exact"])
        outs.append((acts.clone(), r.clone(), d1[0] - d0[0], d1[1] - d0[1]))
    (aa, ra, fa, xa), (ab, rb, _, _) = outs
    print(form, "exact fallbacks after the write:", fa, xa)
    assert fa == 0 and xa == 0
    assert torch.equal(aa, ab)
    assert torch.equal(ra, rb)


def test_greedy_adaptive_band_on_budget_jumps(torch_gpu):
    """MDR_OPT_GQ_ADAPTIVE on the regular-steps signal (a budget jump at every step edge,
    signal_calculator.py:78-98): the ticks whose budget change departs from the last change run the
    three-launch form instead of a band miss.  Three twins over 400 ticks at 1M houses — adaptive, the
    band on every tick, the three-launch form on every tick — give the same actions and rewards bit
    for bit; the adaptive twin skipped the band on some ticks (fewer bins-pass skips recorded than the
    band-only twin) and never fell back to gq_exact."""
    torch = torch_gpu
    from mdr_amd.config import EnvironmentProperties
    from mdr_amd.environment import Environment

    n, T = 1 << 20, 400

    def make():  # (bench.py's C3 configuration, the reference's marl_env_prop.json, regular-steps signal)
        p = EnvironmentProperties.from_json(os.path.join(os.path.dirname(__file__), "golden", "marl_env_prop.json"))
        p.cluster_prop.nb_agents = n
        p.power_grid_prop.signal_properties.mode = "regular_steps"
        return Environment(p, rng=random.Random(4), population="synthetic", seed=1234)

    envs = [make() for _ in range(3)]
    envs[0].shard.set_option("gq_adaptive", 1)
    envs[1].shard.set_option("gq_adaptive", 0)
    envs[2].shard.set_option("gq_band", 0)
    outs = []
    for e in envs:
        b0, g0 = e.shard.greedy_band(), e.shard.greedy_diag()
        acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
        r = e.greedy_rollout(T, actions=acts)[1]
        b1, g1 = e.shard.greedy_band(), e.shard.greedy_diag()
        outs.append((acts, r, b1["skips"] - b0["skips"], g1["fallbacks"] - g0["fallbacks"]))
    print("band skips (adaptive, band only):", outs[0][2], outs[1][2], "fallbacks:", [o[3] for o in outs])
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        assert torch.equal(outs[0][1], o[1])
    assert outs[0][2] < outs[1][2]
    assert outs[0][3] == 0
