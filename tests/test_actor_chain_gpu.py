"""The general MA-PPO actor (row P): the reference Actor takes any ``actor_layers`` list and any obs
width (server/app/core/agents/trainables/network.py:14-33; norm.py:50-66 for the obs row), so the
device actor must too.  Layouts the fused kernel (two hidden layers <= 128 wide, <= 128 feature
slots, weight planes within a CU's LDS) cannot take run the layer chain: k_obs -> k_dense per
hidden layer (split-bf16 MFMA) -> k_actor_head (output layer, softmax, sampling, ON counts).

Checks per layout and precision: which path runs (DeviceActor.fused()), the obs rows == the
standalone obs kernel, probabilities vs torch fp32 on the same rows (fp32 4e-6, bf16x3 1e-4,
bf16 3e-2), prob == probs[action], non-saturated probabilities (golden_util.calibrated_actor), the
graph-captured rollout == the select_actions / step_tensor loop, and the common penalty modes
through DeviceActor.rollout against the oracle's rewards on the same actions."""
import random

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu

ATOL = {"fp32": 4e-6, "fp32_bf16": 4e-6, "bf16x3": 1e-4, "bf16": 3e-2}

# (env overrides, actor_layers, runs fused?)
LAYOUTS = {
    # message_prop thermal + hvac with 10 neighbours: 120 features in 132 slots (> 128)
    "msg_thermal_hvac": ({"cluster_prop.message_prop.thermal": True, "cluster_prop.message_prop.hvac": True},
                         (100, 100), False),
    "three_layers": ({}, (64, 64, 64), False),
    "wide_256": ({}, (256, 256), False),
    "one_layer": ({}, (48,), False),
    # 88 features (KS1 = 4): bf16x3 and the fp16-split fp32 form fit the fused kernel, the three-way
    # bf16 fp32 form's three weight planes do not
    "ks1_4": ({"cluster_prop.message_prop.hvac": True, "state_prop.hvac": True, "state_prop.solar_gain": True,
               "state_prop.thermal": True}, (100, 100), None),
    "default": ({}, (100, 100), True),
}


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _env(n, extra, seed=5, pen="individual_L2"):
    from mdr_amd.environment import Environment

    ov = {"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "sinusoidals",
          "reward_prop.penalty_props.mode": pen}
    ov.update(extra)
    return Environment(gu.props_from_overrides(ov), rng=random.Random(seed))


def _warm(env, torch, ticks=5, seed=7):
    rs = np.random.RandomState(seed)
    for _ in range(ticks):
        env.step_tensor(torch.from_numpy(rs.randint(0, 2, env.n_local).astype(np.uint8)).to("cuda"))


@pytest.mark.parametrize("precision", ["fp32", "fp32_bf16", "bf16x3", "bf16"])
@pytest.mark.parametrize("layout", sorted(LAYOUTS))
def test_actor_layouts_vs_torch(torch_gpu, layout, precision):
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    extra, layers, fused = LAYOUTS[layout]
    n = 3001
    env = _env(n, extra)
    _warm(env, torch)
    F = env.obs_spec().n_feat
    ref_obs = env.obs_tensor().clone()
    actor = gu.calibrated_actor(F, ref_obs.abs().amax(0).double().cpu().numpy(), seed=5, layers=layers).to("cuda")
    if precision == "fp32_bf16":  # (the fp32 precision in its three-way bf16 form)
        da = DeviceActor(env, actor, precision="fp32", fp32_form="bf16_split3")
    else:
        da = DeviceActor(env, actor, precision=precision)
    want_fused = fused if fused is not None else precision != "fp32_bf16"
    assert da.fused() == want_fused
    probs = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    obs = torch.empty((n, F), dtype=torch.float32, device="cuda")
    act, prob = da.select_actions(probs=probs, obs_out=obs, count_next=False)
    assert torch.equal(obs, ref_obs)  # the rows the network read == the standalone obs kernel's
    with torch.no_grad():
        tp = actor(obs).cpu().numpy()
    p = probs.cpu().numpy()
    err = float(np.abs(p - tp).max())
    print(f"{layout} {precision} ({'fused' if want_fused else 'chain'}): max |p - p_torch| = {err:.3g}")
    assert err < ATOL[precision], err
    a = act.cpu().numpy()
    np.testing.assert_array_equal(prob.cpu().numpy(), p[np.arange(n), a])
    gu.assert_not_saturated(tp[:, 1], a)


@pytest.mark.parametrize("layout,T", [("three_layers", 6), ("msg_thermal_hvac", 6), ("three_layers", 1),
                                      ("default", 6)])
def test_chain_rollout_equals_loop(torch_gpu, layout, T):
    """DeviceActor.rollout's captured graph (actor -> step per tick), launched three times (the
    first launch after capture, then two replays), == select_actions / step_tensor, with the counts
    of the sampled actions from k_actor_head (the chain) or k_actor (default: the fused kernel).
    r04 ran the chain uncaptured because its replays read counts of ~1e14 W in ticks 0-1: the
    graph's leading hipMemsetAsync node wrote host stack addresses into the count slabs on every
    replay after the first (ROCm 7.2; tools/chain_bisect.py, tools/graph_memset_repro.hip).  The
    slabs are now zeroed by a kernel node; graph_info asserts that every call replayed the graph."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    extra, layers, _ = LAYOUTS[layout]
    n = 2049
    env_a, env_b = _env(n, extra, 8), _env(n, extra, 8)
    m = env_a.obs_tensor().abs().amax(0).double().cpu().numpy()
    actor = gu.calibrated_actor(env_a.obs_spec().n_feat, m, seed=2, layers=layers).to("cuda")
    da, db = DeviceActor(env_a, actor), DeviceActor(env_b, actor)
    assert da.fused() == (layout == "default")
    rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
    acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    probs = torch.empty((T, n), dtype=torch.float32, device="cuda")
    g0 = env_a.shard.graph_info()
    for rep in range(3):
        da.rollout(T, rewards=rew, actions=acts, probs=probs)
        gi = env_a.shard.graph_info()
        assert gi["actor_launches"] == g0["actor_launches"] + rep + 1, gi
        assert gi["actor_graphs"] == 1, gi
        for t in range(T):
            a, p = db.select_actions(count_next=True)
            r = env_b.step_tensor(a)
            assert torch.equal(a, acts[t]) and torch.equal(p, probs[t]) and torch.equal(r, rew[t]), (rep, t)
    for k in ("t_air", "t_mass", "hvac"):
        assert torch.equal(getattr(env_a.shard, k), getattr(env_b.shard, k)), k
    gu.assert_not_saturated(probs.cpu().numpy(), acts.cpu().numpy())


@pytest.mark.parametrize("pen", ["common_L2", "common_max_error", "mixture"])
def test_actor_rollout_common_penalties_vs_oracle(torch_gpu, pen):
    """DeviceActor.rollout under the common penalty modes (rewards_calculator.py:29-203): the
    rewards of the sampled actions == the oracle stepping the same actions (rtol 1e-9; the cluster
    penalty is reduced in blocked order, the reference adds house by house)."""
    from mdr_amd.actor import DeviceActor
    from oracle import env_np as O

    torch = torch_gpu
    n, T = 1000, 8
    ov = {"reward_prop.penalty_props.alpha_common_max": 0.5}
    env = _env(n, ov, 31, pen=pen)
    props = env.init_props
    ora = O.OracleEnv(props, random.Random(31))
    m = env.obs_tensor().abs().amax(0).double().cpu().numpy()
    da = DeviceActor(env, gu.calibrated_actor(env.obs_spec().n_feat, m, seed=4).to("cuda"))
    acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    R = da.rollout(T, actions=acts).cpu().numpy()
    A = acts.cpu().numpy().astype(bool)
    for t in range(T):
        _, rr = ora.step(A[t])
        np.testing.assert_allclose(R[t], rr, rtol=1e-9, atol=1e-12, err_msg=f"t={t}")
    assert 0 < A.sum() < A.size
