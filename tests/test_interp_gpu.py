"""Row a10 on the GPU: the interpolated base power (k_interp_values / k_interp_sum through the C ABI)
against the reference PowerInterpolator's values (tests/golden/interp.npz, bit-exact) and the
oracle, and windowed rollouts in interpolation mode against the per-step API.

End-to-end trajectories in interpolation mode (dict API and obs vectors vs the reference) run in
tests/test_env_parity_gpu.py (gu.TRAJ_NAMES holds traj_interp_*); the sharded path in
tests/test_distributed_gpu.py / test_distributed_gloo.py."""
import json
import random

import numpy as np
import pytest

import golden_util as gu
from oracle import interp_np as IN

pytestmark = pytest.mark.gpu


def _grids():
    d = gu.load("interp.npz")
    with open(gu.path("interp_parameters_dict.json")) as f:
        params = json.load(f)
    keys = [str(k) for k in d["keys"]]
    return d, [np.asarray(params[k], np.float64) for k in keys]


def test_interp_values_match_reference_points():
    """Each golden point as one house (ratio denominators 1, target 0, so the point's coordinates
    are the house's state exactly), one k_interp_values launch per point: bit-exact."""
    import torch

    from mdr_amd.environment import Environment

    d, grids = _grids()
    raw = d["raw"]
    M = raw.shape[0]
    env = Environment(gu.props_from_overrides({"cluster_prop.nb_agents": M,
                                               "power_grid_prop.signal_properties.mode": "flat"}),
                      rng=random.Random(1), population="synthetic", seed=2)
    sh = env.shard
    table = np.load(gu.interp_table_path())
    sh.interp_load(grids, table, (1.0, 1.0, 1.0, 1.0))
    dev = sh.device
    for k, col in (("ua", 0), ("cm", 1), ("ca", 2), ("hm", 3), ("t_air", 4), ("t_mass", 5)):
        getattr(sh, k).copy_(torch.from_numpy(raw[:, col].copy()).to(dev))
    sh.target.zero_()
    # HVAC_power is a nearest axis: give each house a capacity class with the point's nearest index
    caps = list(env._cap_values)
    hv = grids[7]
    near = [int(np.argmin(np.abs(hv - min(max(v, hv.min()), hv.max())))) for v in raw[:, 7]]
    cls_for = {}
    for ci, c in enumerate(caps):
        cls_for.setdefault(int(np.argmin(np.abs(hv - min(max(c, hv.min()), hv.max())))), ci)
    assert set(near) <= set(cls_for), "the capacity table must reach every HVAC_power index"
    sh.cap_idx.copy_(torch.tensor([cls_for[i] for i in near], dtype=torch.uint8, device=dev))
    vals = torch.empty(M, dtype=torch.float64, device=dev)
    for m in range(M):
        sh.interp_values(torch.tensor([m], dtype=torch.int64, device=dev), raw[m, 6], raw[m, 8], raw[m, 9],
                         vals[m:m + 1])
    got = vals.cpu().numpy()
    np.testing.assert_array_equal(got, d["value"])


def test_interp_sum_and_sharded_slots_vs_oracle():
    """A sampled base power (ids with repeats, out-of-shard ids give 0) == the oracle's ordered sum."""
    import torch

    from mdr_amd.environment import Environment

    d, grids = _grids()
    n = 5000
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "flat"})
    env = Environment(props, rng=random.Random(1), population="synthetic", seed=2)
    sh = env.shard
    hp = props.cluster_prop.house_prop
    table = np.load(gu.interp_table_path())
    cfg = (hp.Ua, hp.Cm, hp.Ca, hp.Hm)
    sh.interp_load(grids, table, cfg)
    for _ in range(5):
        env.step_tensor(None, action_mode="random", lookahead="random")
    rs = np.random.RandomState(3)
    ids = rs.randint(0, n, 100).tolist() + [n + 5, -1]  # two ids outside this shard
    dev = sh.device
    vals = torch.empty(len(ids), dtype=torch.float64, device=dev)
    sh.interp_values(torch.tensor(ids, dtype=torch.int64, device=dev), 31.3, 51234.0, 200.0, vals)
    out = torch.empty(1, dtype=torch.float64, device=dev)
    sh.interp_sum(vals, n / 100.0, out)
    st, prm = sh.host_state(), sh.host_params()
    o = IN.OracleInterp(grids, table, *cfg)
    caps = np.asarray(env._cap_values)[prm["cap_idx"]]
    ref = []
    for j in ids:
        if 0 <= j < n:
            x = o.house_point(prm["ua"][j], prm["cm"][j], prm["ca"][j], prm["hm"][j], st["T"][j], st["Tm"][j],
                              prm["target"][j], 31.3, caps[j], 51234.0, 200.0)
            ref.append(o.point(x))
        else:
            ref.append(0.0)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.array(ref))
    b = 0.0
    for v in ref:
        b += v
    assert float(out.item()) == b * (n / 100.0)


@pytest.mark.parametrize("mode", ["random", "buffer"])
def test_interp_rollout_equals_steps(mode):
    """Windowed rollouts (driver_window stops at every interpolating grid step) == step_tensor."""
    import torch

    from mdr_amd.environment import Environment

    n, T = 4099, 70
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals",
                                     gu.BPP + "mode": "interpolation", gu.BPP + "interp_update_period": 40,
                                     gu.BPP + "interp_nb_agents": 64})
    a = Environment(props, rng=random.Random(9), population="synthetic", seed=4)
    b = Environment(props, rng=random.Random(9), population="synthetic", seed=4)
    b.shard.set_option("window_thermal", 0)  # MDR_THERMAL_EXACT: the interpolated signal reads T bit for bit
    acts = torch.from_numpy(np.random.RandomState(5).randint(0, 2, (T, n)).astype(np.uint8)).to("cuda")
    rew_a, sig = [], []
    for t in range(T):
        if mode == "random":
            r = a.step_tensor(None, action_mode="random", lookahead="random")
        else:
            r = a.step_tensor(acts[t])
        rew_a.append(r.clone())
        sig.append(float(a.power_grid.current_signal))
    rew_b = b.rollout(T, actions=acts if mode == "buffer" else None, action_mode=mode)
    assert torch.equal(torch.stack(rew_a), rew_b)
    assert float(b.power_grid.current_signal) == sig[-1]
    assert a.power_grid.interp.base == b.power_grid.interp.base
    sa, sb = a.shard.host_state(), b.shard.host_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k])


def test_deepcopy_interpolation_env_shares_rng():
    """TrainingManager.test deep-copies the env (training_manager.py:269).  In interpolation mode
    the grid's Interpolator holds the generator — here the `random` module itself, the reference's
    global random, which copy.deepcopy cannot copy: the copy must share it (not fork it), start from
    the same device state, and step exactly like the original from the same RNG state."""
    import copy

    import torch

    from mdr_amd.environment import Environment

    n = 3001
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals",
                                     gu.BPP + "mode": "interpolation", gu.BPP + "interp_update_period": 8,
                                     gu.BPP + "interp_nb_agents": 32})
    random.seed(11)
    env = Environment(props, rng=random, population="synthetic", seed=3)
    for _ in range(5):
        env.step_tensor(None, action_mode="random", lookahead="random")
    twin = copy.deepcopy(env)
    assert twin.rng is env.rng is random
    assert twin.power_grid.interp.rng is env.power_grid.interp.rng
    s0, s1 = env.shard.host_state(), twin.shard.host_state()
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k])
    acts = torch.from_numpy(np.random.RandomState(2).randint(0, 2, (12, n)).astype(np.uint8)).to("cuda")
    out = []
    for e in (env, twin):  # the same RNG state for each: identical trajectories
        random.seed(77)
        out.append(torch.stack([e.step_tensor(acts[t]).clone() for t in range(12)]))
        out.append(float(e.power_grid.current_signal))
    assert torch.equal(out[0], out[2])
    assert out[1] == out[3]
    s0, s1 = env.shard.host_state(), twin.shard.host_state()
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k])
