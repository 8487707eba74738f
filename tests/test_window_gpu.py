"""Temporally blocked rollouts (k_step_window: K ticks per launch, the FSM run ahead for each
tick's cluster power) against the one-tick path and against the oracle.

Two per-tick thermal forms (mdr.h MDR_OPT_WINDOW_THERMAL):
* EXACT — the reference's expression in its operation order: bit-identical to the one-tick kernels,
  which are pinned to the reference goldens (test_env_parity_gpu.py), so `==` carries the parity over;
* AFFINE (the default) — the same update as a per-house affine transition formed once per window:
  FSM / ON masks / P bit-exact, temperatures within 1e-11 relative of the exact form over a window
  and within 1e-9 over 2,000 ticks (north star: 1e-5), rewards alike.
The oracle checks replay the exact in-kernel random actions (tests/philox_np.py), so the benched
action source and form are oracle-checked.
"""
import random

import numpy as np
import pytest

import golden_util as gu
import philox_np as PX
from oracle import env_np as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


# affine vs exact thermal form: the reference's own expression cancels terms of ~5,000 K to a
# ~293 K result, so the two rounding sequences part by ~1e-12 K per tick (measured: 9e-11 K, 5e-12
# relative, after 100 ticks); north star: 1e-5
AFFINE_T_RTOL = 1e-10     # temperatures, within a rollout of <= 131 ticks
AFFINE_R_RTOL, AFFINE_R_ATOL = 1e-9, 1e-10  # rewards -(x^2 + s): relative error grows as x -> 0
AFFINE_LONG_RTOL = 1e-8   # temperatures over 2,000 ticks


def _pair(n, seed=3, pop="synthetic", extra=None, thermal=None):
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    ov = {"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "sinusoidals"}
    ov.update(extra or {})
    props = gu.props_from_overrides(ov)
    e1 = Environment(props, rng=random.Random(seed), population=pop, seed=77)
    e2 = Environment(props, rng=random.Random(seed), population=pop, seed=77)
    if thermal is not None:
        for e in (e1, e2):
            e.shard.set_option("window_thermal", {"exact": L.THERMAL_EXACT, "affine": L.THERMAL_AFFINE}[thermal])
    return e1, e2


def _close_state(torch, e1, e2, rtol):
    """Integer state and P equal, temperatures within rtol (the two thermal forms)."""
    torch.cuda.synchronize()
    s1, s2 = e1.shard.host_state(), e2.shard.host_state()
    for k in ("on", "lock", "sso"):
        np.testing.assert_array_equal(s1[k], s2[k], err_msg=k)
    for k in ("T", "Tm"):
        np.testing.assert_allclose(s1[k], s2[k], rtol=rtol, atol=0, err_msg=k)
    assert e1._cluster_power() == e2._cluster_power()


def _same_state(torch, e1, e2):
    torch.cuda.synchronize()
    s1, s2 = e1.shard.host_state(), e2.shard.host_state()
    for k in s1:
        np.testing.assert_array_equal(s1[k], s2[k], err_msg=k)
    assert e1._cluster_power() == e2._cluster_power()


@pytest.mark.parametrize("n,ticks,win", [(1, 5, 32), (2, 33, 32), (257, 40, 7), (4099, 65, 32),
                                         (20011, 64, 16), (131072, 50, 32)])
@pytest.mark.parametrize("mode", ["random", "always_on", "buffer"])
@pytest.mark.parametrize("thermal", ["exact", "affine"])
@pytest.mark.parametrize("use_graph", [False, True])
def test_window_equals_one_tick(torch_gpu, n, ticks, win, mode, thermal, use_graph):
    """Windowed rollout (direct launches with kernel-argument drivers, or a replayed graph) vs the
    one-launch-per-tick rollout: EXACT bit for bit (rewards, state, P); AFFINE with the masks,
    counters and P bit for bit, temperatures within AFFINE_T_RTOL, rewards within AFFINE_R_*."""
    torch = torch_gpu
    e1, e2 = _pair(n, thermal=thermal)
    e1.shard.set_rollout_window(win)
    e2.shard.set_rollout_window(0)
    acts = None
    if mode == "buffer":
        g = torch.Generator(device="cuda").manual_seed(n)
        acts = (torch.rand((ticks, n), device="cuda", generator=g) < 0.5).to(torch.uint8)
    for rep in range(2):  # second call replays the cached graphs
        r1 = e1.rollout(ticks, actions=acts, action_mode=mode, use_graph=use_graph)
        r2 = e2.rollout(ticks, actions=acts, action_mode=mode)
        if thermal == "exact":
            np.testing.assert_array_equal(r1.cpu().numpy(), r2.cpu().numpy())
            _same_state(torch, e1, e2)
        else:
            np.testing.assert_allclose(r1.cpu().numpy(), r2.cpu().numpy(), rtol=AFFINE_R_RTOL, atol=AFFINE_R_ATOL)
            _close_state(torch, e1, e2, AFFINE_T_RTOL)


@pytest.mark.parametrize("n", [4099, 65536])
def test_affine_form_long_run(torch_gpu, n):
    """2,000 ticks (63 windows) of the default AFFINE form against the EXACT form from the same
    state: masks, counters and P exact every call; temperatures and rewards within
    AFFINE_LONG_RTOL at the end (the slow thermal mode keeps per-tick differences, ~1e-13 K)."""
    torch = torch_gpu
    e1, e2 = _pair(n)
    from mdr_amd import _lib as L

    e2.shard.set_option("window_thermal", L.THERMAL_EXACT)
    worst = 0.0
    for c in range(10):
        r1 = e1.rollout(200, action_mode="random")
        r2 = e2.rollout(200, action_mode="random")
        _close_state(torch, e1, e2, AFFINE_LONG_RTOL)
        d = (r1 - r2).abs().max().item()
        worst = max(worst, d)
        assert d <= 1e-8, (c, d)
    s1, s2 = e1.shard.host_state(), e2.shard.host_state()
    rel = float(np.max(np.abs(s1["T"] - s2["T"]) / np.abs(s2["T"])))
    print(f"n={n}: after 2000 ticks max rel |T_affine - T_exact| = {rel:.3g}, max |dr| = {worst:.3g}")


C2_TICKS = 10000  # 64k houses x T = 10,000


def test_affine_form_c2_horizon_vs_exact(torch_gpu):
    """C2's whole horizon, 65,536 houses x 10,000 ticks (313 windows), of the default AFFINE form
    against the EXACT form (bit-identical to the one-tick kernels, which the reference goldens pin):
    ON masks, lockout, seconds-since-off and P `==` after every 1,000-tick call; temperatures and
    rewards within the north star's 1e-5 relative at every call (measured drift printed)."""
    torch = torch_gpu
    from mdr_amd import _lib as L

    e1, e2 = _pair(65536)
    e2.shard.set_option("window_thermal", L.THERMAL_EXACT)
    worst_r = worst_t = 0.0
    for c in range(C2_TICKS // 1000):
        r1 = e1.rollout(1000, action_mode="random")
        r2 = e2.rollout(1000, action_mode="random")
        _close_state(torch, e1, e2, 1e-5)
        rel = ((r1 - r2).abs() / r2.abs().clamp_min(1e-3)).max().item()
        assert rel <= 1e-5, (c, rel)
        worst_r = max(worst_r, rel)
        s1, s2 = e1.shard.host_state(), e2.shard.host_state()
        worst_t = max(worst_t, float(np.max(np.abs(s1["T"] - s2["T"]) / np.abs(s2["T"]))))
    assert e1._tick == e2._tick
    print(f"65,536 x {C2_TICKS} ticks: max rel |T_affine - T_exact| = {worst_t:.3g}, "
          f"max rel reward difference = {worst_r:.3g}")


def test_affine_form_c2_horizon_vs_oracle(torch_gpu):
    """The benched form (AFFINE, random actions) over C2's 10,000-tick horizon against the oracle
    stepping the same Philox actions (4,096 houses, so the NumPy oracle finishes in seconds):
    on / lock / sso and P `==` at the last tick, T, Tm and the last tick's rewards within 1e-5
    relative (north star)."""
    from mdr_amd.environment import Environment

    n, seed = 4096, 4
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(seed), seed=1234)
    ora = O.OracleEnv(props, random.Random(seed))
    tick0 = env._tick
    rows = []
    for c in range(C2_TICKS // 1000):
        rows.append(env.rollout(1000, action_mode="random")[-1].cpu().numpy())
    gids = np.arange(n, dtype=np.uint64)
    for t in range(C2_TICKS):
        o, rr = ora.step(PX.random_actions(1234, gids, tick0 + t))
        if t % 1000 == 999:
            np.testing.assert_allclose(rows[t // 1000], rr, rtol=1e-5, atol=1e-8, err_msg=f"reward t={t}")
    st = env.shard.host_state()
    for k in ("on", "lock", "sso"):
        np.testing.assert_array_equal(st[k], o[k], err_msg=k)
    np.testing.assert_allclose(st["T"], o["T"], rtol=1e-5, atol=0)
    np.testing.assert_allclose(st["Tm"], o["Tm"], rtol=1e-5, atol=0)
    assert env.cluster.current_power_consumption == o["P"]
    rel = float(np.max(np.abs(st["T"] - o["T"]) / np.abs(o["T"])))
    print(f"4,096 x {C2_TICKS} ticks vs the oracle: max rel |T - T_oracle| = {rel:.3g}")


def test_window_options_validated(torch_gpu):
    """mdr_set_option rejects unknown options and out-of-range values (MDR_EARG)."""
    from mdr_amd import _lib as L

    e1, _ = _pair(65)
    with pytest.raises(L.MdrError):
        e1.shard.set_option("window_thermal", 7)
    with pytest.raises(L.MdrError):
        e1.shard.set_option("step_tpw", 9)
    with pytest.raises(L.MdrError):
        L.check(e1.shard.lib.mdr_set_option(e1.shard.ctx, 99, 1), "unknown option")


def test_window_one_row_rewards(torch_gpu):
    """rewards given as ONE row (every tick overwrites it): the last tick's rewards remain."""
    torch = torch_gpu
    e1, e2 = _pair(5001)
    row = torch.empty(5001, dtype=torch.float64, device="cuda")
    e1.rollout(45, action_mode="random", rewards=row)
    full = e2.rollout(45, action_mode="random")
    np.testing.assert_array_equal(row.cpu().numpy(), full[-1].cpu().numpy())
    _same_state(torch, e1, e2)


def test_window_then_steps(torch_gpu):
    """A windowed rollout leaves the env where step_tensor continues from (counts, ticks, P)."""
    torch = torch_gpu
    e1, e2 = _pair(3000, thermal="exact")
    e1.rollout(37, action_mode="random")
    for _ in range(37):
        e2.step_tensor(None, action_mode="random")
    r1 = [e1.step_tensor(None, action_mode="random").clone() for _ in range(5)]
    r2 = [e2.step_tensor(None, action_mode="random").clone() for _ in range(5)]
    np.testing.assert_array_equal(torch.stack(r1).cpu().numpy(), torch.stack(r2).cpu().numpy())
    _same_state(torch, e1, e2)


def test_random_rollout_vs_oracle_replayed_actions(torch_gpu):
    """rollout(action_mode='random') at 65,536 houses x 50 ticks == the oracle stepping the SAME
    Philox actions (restated in NumPy): on/lock/sso exact, temperatures rtol 1e-10, rewards, P."""
    from mdr_amd.environment import Environment

    n, T, seed = 65536, 50, 4
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(seed), seed=1234)
    ora = O.OracleEnv(props, random.Random(seed))
    tick0 = env._tick
    R = env.rollout(T, action_mode="random").cpu().numpy()
    gids = np.arange(n, dtype=np.uint64)
    ones = 0
    for t in range(T):
        a = PX.random_actions(1234, gids, tick0 + t)
        ones += int(a.sum())
        o, rr = ora.step(a)
        np.testing.assert_allclose(R[t], rr, rtol=1e-9, atol=1e-12, err_msg=f"reward t={t}")
    st = env.shard.host_state()
    np.testing.assert_array_equal(st["on"], o["on"])
    np.testing.assert_array_equal(st["lock"], o["lock"])
    np.testing.assert_array_equal(st["sso"], o["sso"])
    np.testing.assert_allclose(st["T"], o["T"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(st["Tm"], o["Tm"], rtol=1e-10, atol=0)
    assert env.cluster.current_power_consumption == o["P"]
    # Bernoulli(0.5): 3.3M draws within 4 sigma
    assert abs(ones / (n * T) - 0.5) < 4 * 0.5 / np.sqrt(n * T)


def test_time_step_kernels_advances_like_rollout(torch_gpu):
    """mdr_time_step_kernels (the bench's per-launch kernel timing) issues the rollout's launch
    sequence directly: one step launch per window, positive time, and the same state and rewards
    as a graph-replayed rollout."""
    torch = torch_gpu
    from mdr_amd import _lib as L

    n, T = 70001, 75
    e1, e2 = _pair(n)
    r1 = torch.empty((T, n), dtype=torch.float64, device="cuda")
    r2 = torch.empty_like(r1)
    ms, launches = e1.shard.time_step_kernels(e1.driver_window(T), None, 0, L.ACT_RANDOM, r1, n)
    e2.rollout(T, action_mode="random", rewards=r2)
    assert launches == -(-T // 32) and ms > 0.0
    torch.cuda.synchronize()
    s1, s2 = e1.shard.host_state(), e2.shard.host_state()
    for k in s1:
        np.testing.assert_array_equal(s1[k], s2[k], err_msg=k)
    assert torch.equal(r1, r2)


@pytest.mark.parametrize("mode", ["random", "buffer"])
def test_rollout_begin_early_count(torch_gpu, mode):
    """mdr_rollout_begin (the first window's count launched before the drivers): Environment.rollout
    uses it, and an early count that the next call does not match (another length, a step in
    between, another first tick) is discarded — every variant equals a twin run without it."""
    torch = torch_gpu
    from mdr_amd import _lib as L

    n = 9001
    e1, e2 = _pair(n)
    m = L.ACT_RANDOM if mode == "random" else L.ACT_BUFFER
    acts = (torch.rand((40, n), device="cuda") < 0.5).to(torch.uint8) if mode == "buffer" else None
    r1 = torch.empty((40, n), dtype=torch.float64, device="cuda")
    r2 = torch.empty_like(r1)

    def roll(env, k, r, begin=True):
        a = None if acts is None else acts[:k]
        if not begin:  # the twin: the same C calls without the early count
            ticks = env.driver_window(k)
            env.shard.rollout(ticks, a, n if a is not None else 0, m, r[:k], n, True)
            env._P_dev_valid = True
        else:
            env.rollout(k, actions=a, action_mode=mode, rewards=r[:k])

    for k in (20, 40, 7):  # consumed early counts (Environment.rollout calls mdr_rollout_begin)
        roll(e1, k, r1)
        roll(e2, k, r2, begin=False)
        _same_state(torch, e1, e2)
        assert torch.equal(r1[:k], r2[:k])
    # unmatched early counts: another length, an intervening step, a stale first tick
    sa = None if acts is None else acts
    e1.shard.rollout_begin(33, e1._tick, sa, n if sa is not None else 0, m)
    roll(e1, 20, r1, begin=False)
    roll(e2, 20, r2, begin=False)
    _same_state(torch, e1, e2)
    assert torch.equal(r1[:20], r2[:20])
    e1.shard.rollout_begin(20, e1._tick, sa, n if sa is not None else 0, m)
    step_a = (torch.rand(n, device="cuda") < 0.5).to(torch.uint8)
    e1.step_tensor(step_a)
    e2.step_tensor(step_a)
    roll(e1, 20, r1, begin=False)
    roll(e2, 20, r2, begin=False)
    _same_state(torch, e1, e2)
    assert torch.equal(r1[:20], r2[:20])
    e1.shard.rollout_begin(20, e1._tick + 5, sa, n if sa is not None else 0, m)
    roll(e1, 20, r1, begin=False)
    roll(e2, 20, r2, begin=False)
    _same_state(torch, e1, e2)
    assert torch.equal(r1[:20], r2[:20])


@pytest.mark.parametrize("deadband", [0.0, 0.5])
@pytest.mark.parametrize("mode", ["random", "always_on", "buffer"])
def test_rollout_direct_kernarg_drivers(torch_gpu, mode, deadband):
    """Environment.rollout's default (direct launches): the first window's count and P-only reduce
    are launched before the drivers exist; the drivers then ride as kernel arguments of the first
    step kernel (k_step_window<..., KA>, the SIMPLE reward or, deadband != 0, the general one) and
    the rest are staged behind the first step kernel.  Calls of 1, 20, 45, 64, 65, 100 and 131
    ticks back to back equal a graph-replayed twin that stages every driver first (rewards, state
    and P compared with ==)."""
    torch = torch_gpu
    from mdr_amd import _lib as L

    n = 9000
    e1, e2 = _pair(n, extra={"cluster_prop.house_prop.deadband": deadband})
    m = {"random": L.ACT_RANDOM, "always_on": L.ACT_ALWAYS_ON, "buffer": L.ACT_BUFFER}[mode]
    T = 131
    acts = (torch.rand((T, n), device="cuda") < 0.5).to(torch.uint8) if mode == "buffer" else None
    r1 = torch.empty((T, n), dtype=torch.float64, device="cuda")
    r2 = torch.empty_like(r1)
    for k in (1, 20, 45, 64, 65, 100, 131):
        a = None if acts is None else acts[:k]
        e1.rollout(k, actions=a, action_mode=mode, rewards=r1[:k])
        ticks = e2.driver_window(k)
        e2.shard.rollout(ticks, a, n if a is not None else 0, m, r2[:k], n, True)
        e2._P_dev_valid = True
        e2.finish_grid_step()
        _same_state(torch, e1, e2)
        assert torch.equal(r1[:k], r2[:k]), k
        assert float(e1.shard.p_dev.item()) == float(e2.shard.p_dev.item())


@pytest.mark.parametrize("start", [(23, 58, 30), (23, 58, 40), (0, 0, 0)])
def test_rollout_fused_call_across_midnight(torch_gpu, start):
    """Environment.rollout's one-C-call sequence (_mdr_host.rollout1: mdr_rollout_begin, the host
    drivers, mdr_rollout) when the window crosses midnight: the first day's ticks come from that
    call, which then leaves the launch to Python (the next day's tables); equal to a
    graph-replayed twin that stages every driver first (rewards, state, P ==).  Starts 22 ticks
    before midnight, exactly 20 ticks before it (the window ends on the last tick of the day), and
    at midnight."""
    import datetime as dt

    torch = torch_gpu
    from mdr_amd import _lib as L

    n = 5000
    e1, e2 = _pair(n)
    for e in (e1, e2):
        e.date_time = e.date_time.replace(hour=start[0], minute=start[1], second=start[2])
    r1 = torch.empty((40, n), dtype=torch.float64, device="cuda")
    r2 = torch.empty_like(r1)
    for k in (40, 20, 33):
        e1.rollout(k, action_mode="random", rewards=r1[:k])
        ticks = e2.driver_window(k)
        e2.shard.rollout(ticks, None, 0, L.ACT_RANDOM, r2[:k], n, True)
        e2._P_dev_valid = True
        e2.finish_grid_step()
        _same_state(torch, e1, e2)
        assert torch.equal(r1[:k], r2[:k]), k
        assert e1.date_time == e2.date_time and e1._tick == e2._tick
        assert float(e1.shard.p_dev.item()) == float(e2.shard.p_dev.item())
