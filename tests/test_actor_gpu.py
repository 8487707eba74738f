"""Fused obs + MA-PPO actor kernel (row P) vs the reference actor and torch fp32.

Reference: Actor.forward (server/app/core/agents/trainables/network.py:29-33) with the MAPPO seed-1
initialisation (mappo.py:41-50), on norm_state_dict vectors (norm.py:178-218); golden
``tests/golden/policy.npz`` (reference probabilities on reference obs vectors).

Tolerances on action probabilities (the kernel's documented precision, mdr.h MDR_PREC_*):
  fp32   (fp16 hi/lo split on the fp16 MFMA, 3 products, per-layer power-of-two weight scales, fp32
         accumulate: the default fp32 form)  atol 1e-6 against torch fp32
  fp32_bf16 (the fp32 precision in its three-way split-bf16 form, 6 products)  atol 1e-6
  bf16x3 (split-bf16 MFMA, fp32 accumulate)  atol 1e-4 against torch fp32 on the same obs
  bf16   (one bf16 product per term)         atol 3e-2
Obs rows: within 2 float32 ulps of the reference (as tests/test_env_parity_gpu.py); bit-identical
to the standalone obs kernel.  Sampling RNG is not part of parity; the sampled
action is checked for consistency (prob == probs[action]) and statistically.
"""
import random

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu

PROB_ATOL = {"fp32": 1e-6, "fp32_bf16": 1e-6, "bf16x3": 1e-4, "bf16": 3e-2}
FP32S = ("fp32", "fp32_bf16")


def device_actor(env, actor, precision):
    """DeviceActor for a test precision: 'fp32_bf16' = precision fp32 in its three-way bf16 form."""
    from mdr_amd.actor import DeviceActor

    if precision == "fp32_bf16":
        return DeviceActor(env, actor, precision="fp32", fp32_form="bf16_split3")
    return DeviceActor(env, actor, precision=precision)
POLICY_CASES = {"c1": ("c1_sin_dbbc", (0, 1, 50)), "wide": ("n30_maxerr_groups_hvacmsg", (0, 50))}


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def ref_actor(torch, case):
    from mdr_amd.actor import make_actor

    d = gu.load("policy.npz")
    n_in = d[f"{case}_fc.0.weight"].shape[1]
    a = make_actor(n_in, 2, [100, 100], seed=None)
    a.load_state_dict({k[len(case) + 1:]: torch.from_numpy(d[k]) for k in d.files
                       if k.startswith(case + "_fc.")})
    return a.to("cuda"), d


def make_env(props, rng_seed, resets=1, **kw):
    from mdr_amd.environment import Environment

    env = Environment(props, rng=random.Random(rng_seed), **kw)
    for _ in range(resets - 1):
        env.reset(return_obs=False)
    return env


@pytest.mark.parametrize("precision", ["fp32", "fp32_bf16", "bf16x3", "bf16"])
@pytest.mark.parametrize("case", sorted(POLICY_CASES))
def test_actor_golden(torch_gpu, case, precision):
    """Reference actor weights + reference trajectory state: obs rows and probabilities."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    actor, pol = ref_actor(torch, case)
    name, ticks = POLICY_CASES[case]
    d, meta = gu.traj(name)
    props = gu.props_from_overrides(meta["overrides"])
    env = make_env(props, meta["seed"], meta["resets"])
    da = device_actor(env, actor, precision)
    N, F = meta["N"], pol[f"{case}_obs"].shape[1]
    ref_obs = pol[f"{case}_obs"].reshape(len(ticks), N, F)
    ref_probs = pol[f"{case}_probs"].reshape(len(ticks), N, 2)
    worst = 0.0
    for t in range(max(ticks) + 1):
        if t in ticks:
            k = ticks.index(t)
            probs = torch.empty((N, 2), dtype=torch.float32, device="cuda")
            obs = torch.empty((N, F), dtype=torch.float32, device="cuda")
            act, prob = da.select_actions(probs=probs, obs_out=obs, count_next=False)
            o = obs.cpu().numpy()
            np.testing.assert_array_max_ulp(o, ref_obs[k], maxulp=2)
            np.testing.assert_array_equal(o, env.obs_tensor().cpu().numpy())  # == standalone obs kernel
            with torch.no_grad():
                tp = actor(obs).cpu().numpy()  # torch fp32 on the identical rows
            p = probs.cpu().numpy()
            err = float(np.abs(p - tp).max())
            worst = max(worst, err)
            assert err < PROB_ATOL[precision], (t, err)
            # (the golden holds the reference's CPU probabilities: torch's CPU and GPU fp32 GEMMs
            # accumulate in other orders, ~1e-7)
            assert np.abs(p - ref_probs[k]).max() < PROB_ATOL[precision] + (1e-6 if precision in FP32S else 1e-5)
            a = act.cpu().numpy()
            np.testing.assert_array_equal(prob.cpu().numpy(), p[np.arange(N), a])
        if t < max(ticks):
            env.step_tensor(torch.from_numpy(d["actions"][t]).to("cuda"))
    print(f"{case} {precision}: max |p - p_torch| = {worst:.3g}")
    assert da.status()["range_faults"] == 0


def scaled_actor(torch, n_in, scale, seed=3):
    from mdr_amd.actor import make_actor

    a = make_actor(n_in, 2, [100, 100], seed=seed)
    with torch.no_grad():
        for p in a.parameters():
            p.mul_(scale)
    return a.to("cuda")


def _forward64(actor, x):
    """The actor's logits in float64 (network.py:29-33 without the softmax)."""
    import torch

    for i, l in enumerate(actor.fc):
        x = torch.nn.functional.linear(x, l.weight.double(), l.bias.double())
        if i + 1 < len(actor.fc):
            x = torch.relu(x)
    return x


@pytest.mark.parametrize("precision", ["fp32", "fp32_bf16", "bf16x3", "bf16"])
@pytest.mark.parametrize("n", [1, 37, 300, 4099])
def test_actor_vs_torch_sizes(torch_gpu, n, precision):
    """Ragged sizes, spread-out logits (weights x3): probabilities vs torch fp32 on the same obs."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = make_env(props, 11)
    rs = np.random.RandomState(n)
    for _ in range(7):
        env.step_tensor(torch.from_numpy(rs.randint(0, 2, n).astype(np.uint8)).to("cuda"))
    F = env.obs_spec().n_feat
    actor = scaled_actor(torch, F, 3.0)
    da = device_actor(env, actor, precision)
    probs = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    obs = torch.empty((n, F), dtype=torch.float32, device="cuda")
    act, prob = da.select_actions(probs=probs, obs_out=obs, count_next=False)
    with torch.no_grad():
        tp = actor(obs).cpu().numpy()
    p = probs.cpu().numpy()
    err = float(np.abs(p - tp).max())
    print(f"n={n} {precision}: max |p - p_torch| = {err:.3g}, p1 spread {tp[:, 1].min():.3f}..{tp[:, 1].max():.3f}")
    if precision in FP32S:
        # fp32-faithful: no further from the float64 forward than torch's own fp32 GEMMs are (other
        # accumulation orders; at weights x3 the logits reach tens, so both sit at a few 1e-7 .. 1e-6)
        with torch.no_grad():
            p64 = torch.softmax(_forward64(actor, obs.double()), 1).cpu().numpy()
        e_ours, e_torch = float(np.abs(p - p64).max()), float(np.abs(tp - p64).max())
        print(f"  vs float64: ours {e_ours:.3g}, torch fp32 {e_torch:.3g}")
        assert e_ours <= 2.0 * e_torch + 2e-7
        assert err < 4e-6
    else:
        assert err < PROB_ATOL[precision]
    a = act.cpu().numpy()
    assert set(np.unique(a)) <= {0, 1}
    np.testing.assert_array_equal(prob.cpu().numpy(), p[np.arange(n), a])


LAYOUTS = {
    # 2 neighbours: 18 features, 20 slots -> one k-step of 32, run as KS1 = 2 with a zero k-step
    "ks1_padded": {"cluster_prop.agents_comm_prop.max_nb_agents_communication": 2},
    # every own-state feature + hvac messages: 88 features, 100 slots -> KS1 = 4
    "ks1_4": {"cluster_prop.message_prop.hvac": True, "state_prop.hvac": True, "state_prop.solar_gain": True,
              "state_prop.thermal": True},
}


@pytest.mark.parametrize("precision", ["fp32", "fp32_bf16", "bf16x3"])
@pytest.mark.parametrize("layout", sorted(LAYOUTS))
def test_actor_layer1_ksteps(torch_gpu, layout, precision):
    """The layer-1 k-step instantiations at their edges (mdr_actor.hip KS1): probabilities vs torch
    fp32 on the same obs rows, at 3,001 houses (a ragged last tile)."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    n = 3001
    ov = {"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "sinusoidals"}
    ov.update(LAYOUTS[layout])
    env = make_env(gu.props_from_overrides(ov), 5)
    rs = np.random.RandomState(7)
    for _ in range(5):
        env.step_tensor(torch.from_numpy(rs.randint(0, 2, n).astype(np.uint8)).to("cuda"))
    F = env.obs_spec().n_feat
    assert F == {"ks1_padded": 18, "ks1_4": 88}[layout]
    # (the obs normalisation folded into layer 1: probabilities away from saturation, so the
    # check compares real numbers — r03's scaled actor saturated at 88 features)
    actor = gu.calibrated_actor(F, env.obs_tensor().abs().amax(0).double().cpu().numpy(), seed=5).to("cuda")
    probs = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    obs = torch.empty((n, F), dtype=torch.float32, device="cuda")
    da = device_actor(env, actor, precision)
    # (ks1_4 in the three-way bf16 fp32 form: three planes of W1 (7 x 4 k-steps) and W2 (7 x 4) are
    # 168 KiB, more than a CU's LDS, so that layout runs the layer chain, tests/test_actor_chain_gpu.py;
    # the fp16-split form has two planes, like bf16x3, and runs fused)
    assert da.fused() == (layout != "ks1_4" or precision != "fp32_bf16")
    da.select_actions(probs=probs, obs_out=obs, count_next=False)
    with torch.no_grad():
        tp = actor(obs).cpu().numpy()
    err = float(np.abs(probs.cpu().numpy() - tp).max())
    print(f"{layout} {precision}: max |p - p_torch| = {err:.3g}")
    assert err < (4e-6 if precision in FP32S else PROB_ATOL[precision])
    gu.assert_not_saturated(tp[:, 1])


@pytest.mark.parametrize("precision", ["fp32", "fp32_bf16", "bf16x3", "bf16"])
def test_actor_default_layout_form_equals_generic(torch_gpu, precision):
    """The k_actor form specialised for the reference's default obs layout (mdr_actor.hip DEF: its
    layout fixed at compile time, 12 / 16 waves per block) == the generic form on the same inputs,
    bit for bit: probabilities, actions, chosen probabilities and obs rows (MDR_OPT_ACTOR_GENERIC
    switches between them; the ON counts of the new actions come from the same FSM code and are
    checked on the default form by test_actor_count_next_equals_power_counts)."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    n = 40_000
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = make_env(props, 13)
    rs = np.random.RandomState(3)
    for _ in range(4):
        env.step_tensor(torch.from_numpy(rs.randint(0, 2, n).astype(np.uint8)).to("cuda"))
    F = env.obs_spec().n_feat
    actor = gu.calibrated_actor(F, env.obs_tensor().abs().amax(0).double().cpu().numpy(), seed=9).to("cuda")
    da = device_actor(env, actor, precision)
    res = []
    for generic in (0, 1):
        env.shard.set_option("actor_generic", generic)
        probs = torch.empty((n, 2), dtype=torch.float32, device="cuda")
        obs = torch.empty((n, F), dtype=torch.float32, device="cuda")
        act, prob = da.select_actions(probs=probs, obs_out=obs, count_next=False)
        res.append((probs, obs, act.clone(), prob.clone()))
    env.shard.set_option("actor_generic", 0)
    for k, (x, y) in enumerate(zip(*res)):
        assert torch.equal(x, y), k
    gu.assert_not_saturated(res[0][0][:, 1].cpu().numpy(), res[0][2].cpu().numpy())


def test_actor_sampling_statistics(torch_gpu):
    """Categorical sampling: the fraction of houses turning on matches the mean probability."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    n = 200_000
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = make_env(props, 5, population="synthetic", seed=77)
    actor = scaled_actor(torch, env.obs_spec().n_feat, 1.0)
    da = DeviceActor(env, actor)
    probs = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    act, _ = da.select_actions(probs=probs, count_next=False)
    p1 = probs[:, 1].double()
    mean, var = float(p1.mean()), float((p1 * (1 - p1)).sum())
    ones = float(act.double().sum())
    assert abs(ones - mean * n) < 6 * var ** 0.5 + 1, (ones, mean * n, var ** 0.5)


def test_actor_count_next_equals_power_counts(torch_gpu):
    """select_actions(count_next) + step_tensor == the same actions through mdr_power_counts."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    n = 5000
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env_a, env_b = make_env(props, 21), make_env(props, 21)
    actor = scaled_actor(torch, env_a.obs_spec().n_feat, 2.0)
    da = DeviceActor(env_a, actor)
    for t in range(6):
        act, _ = da.select_actions(count_next=True)
        ra = env_a.step_tensor(act).clone()
        rb = env_b.step_tensor(act.clone()).clone()
        torch.testing.assert_close(ra, rb, rtol=0, atol=0)
        for k in ("t_air", "t_mass", "hvac"):
            assert torch.equal(getattr(env_a.shard, k), getattr(env_b.shard, k)), (t, k)


def test_actor_rollout_equals_loop(torch_gpu):
    """DeviceActor.rollout (one hipGraph: actor -> step per tick) == select_actions/step_tensor loop."""
    from mdr_amd.actor import DeviceActor

    torch = torch_gpu
    n, T = 3001, 12
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env_a, env_b = make_env(props, 8), make_env(props, 8)
    actor = scaled_actor(torch, env_a.obs_spec().n_feat, 2.0)
    da, db = DeviceActor(env_a, actor), DeviceActor(env_b, actor)
    rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
    acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    probs = torch.empty((T, n), dtype=torch.float32, device="cuda")
    da.rollout(T, rewards=rew, actions=acts, probs=probs)
    for t in range(T):
        a, p = db.select_actions(count_next=True)
        r = env_b.step_tensor(a)
        assert torch.equal(a, acts[t]), t
        assert torch.equal(p, probs[t]), t
        assert torch.equal(r, rew[t]), t
    for k in ("t_air", "t_mass", "hvac"):
        assert torch.equal(getattr(env_a.shard, k), getattr(env_b.shard, k)), k
    # a second rollout replays the cached graph with the next ticks' drivers
    da.rollout(T, rewards=rew, actions=acts, probs=probs)
    for t in range(T):
        a, p = db.select_actions(count_next=True)
        r = env_b.step_tensor(a)
        assert torch.equal(a, acts[t]) and torch.equal(r, rew[t]), t


@pytest.mark.parametrize("precision", FP32S)
def test_actor_fp32_rollout_equals_loop(torch_gpu, precision):
    """The fp32-faithful precision (both forms) through the fused rollout graph == its select_actions
    / step_tensor loop (the same kernel in both)."""
    torch = torch_gpu
    n, T = 2049, 6
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env_a, env_b = make_env(props, 8), make_env(props, 8)
    actor = scaled_actor(torch, env_a.obs_spec().n_feat, 2.0)
    da, db = device_actor(env_a, actor, precision), device_actor(env_b, actor, precision)
    rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
    acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    da.rollout(T, rewards=rew, actions=acts)
    for t in range(T):
        a, _ = db.select_actions(count_next=True)
        r = env_b.step_tensor(a)
        assert torch.equal(a, acts[t]) and torch.equal(r, rew[t]), t


def test_actor_fp16_split_range(torch_gpu):
    """The fp16-split fp32 form beyond fp16's range: houses off for ~34 years (sso saturated at
    2^30 - 1 s: a seconds-since-off ratio of ~2.7e7, beyond fp16's 65504, in their own rows and their
    ring neighbours' messages) make k_actor compute their tiles' logits in scalar fp32 from the raw
    weights (mdr_actor_status 'exact'); every house's probabilities then match torch fp32 within the
    fp32 tolerance, as the three-way bf16 form's do.  A normal state needs no such tile."""
    torch = torch_gpu
    n = 3001
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = make_env(props, 5)
    for _ in range(3):
        env.step_tensor(torch.zeros(n, dtype=torch.uint8, device="cuda"))
    F = env.obs_spec().n_feat
    actor = gu.calibrated_actor(F, env.obs_tensor().abs().amax(0).double().cpu().numpy(), seed=4).to("cuda")
    for big in (False, True):
        if big:  # houses 100..131 off for ~34 years (hvac bits 0-29 saturated)
            env.shard.hvac[100:132] = 0x3FFFFFFF
        obs = env.obs_tensor().clone()
        assert (float(obs[100:132].abs().max()) > 65504.0) == big
        with torch.no_grad():
            tp = actor(obs).cpu().numpy()
        for precision in FP32S:
            da = device_actor(env, actor, precision)
            da.status()  # (clear)
            probs = torch.empty((n, 2), dtype=torch.float32, device="cuda")
            da.select_actions(probs=probs, count_next=False)
            st = da.status()
            p = probs.cpu().numpy()
            assert np.all(np.isfinite(p)) and np.abs(p - tp).max() < 4e-6, (big, precision, np.abs(p - tp).max())
            assert st["range_faults"] == 0, st
            if precision == "fp32":
                assert st["kernel_prec"] == 4 and (st["exact"] >= 1) == big, st
            else:
                assert st["kernel_prec"] == 6 and st["exact"] == 0, st
