"""The step kernels' shared-reciprocal division (mdr_device.h `recip`/`div_by`) must be
bit-identical to the IEEE `/` operator inside its guarded operand range ([2^-300, 2^300])."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_shared_reciprocal_division_is_exact():
    import torch

    from mdr_amd import _lib as L

    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(7)
    n = 1 << 24
    total = 0
    for rep in range(6):
        if rep < 4:  # log-uniform magnitudes, random signs, across the guarded range
            ea = (torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 600 - 300)
            eb = (torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 600 - 300)
            a = torch.exp2(ea) * torch.where(torch.rand(n, device="cuda", generator=g) < 0.5, -1.0, 1.0).double()
            b = torch.exp2(eb) * torch.where(torch.rand(n, device="cuda", generator=g) < 0.5, -1.0, 1.0).double()
        else:  # the step's own operand scales (Ca ~ 1e6, Hm ~ 3e3, Ua ~ 1, temperatures ~ 300 K)
            a = (torch.rand(n, device="cuda", generator=g, dtype=torch.float64) - 0.5) * 1e7
            b = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 2e6 + 0.5
        mism = torch.zeros(1, dtype=torch.int64, device="cuda")
        L.check(lib.mdr_div_check(a.data_ptr(), b.data_ptr(), n, mism.data_ptr(), 0))
        torch.cuda.synchronize()
        total += int(mism.item())
    assert total == 0


@pytest.mark.parametrize("tpw", [0, -1])
def test_step_fastdiv_bit_identical(tpw):
    """The shared-reciprocal division (default) and the IEEE operator everywhere
    (MDR_OPT_FASTDIV = 0) produce bit-identical trajectories, in k_step_t (tpw 0) and in the
    default per-tick kernel."""
    import torch

    import golden_util as gu
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 100_003,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    envs = []
    for fast in (0, 1):
        e = Environment(props, rng=random.Random(2), population="synthetic", seed=3)
        e.shard.set_option("fastdiv", fast)
        e.shard.set_option("step_tpw", tpw)
        envs.append(e)
    for t in range(40):
        rs = [e.step_tensor(None, action_mode="random", lookahead="random").clone() for e in envs]
        assert torch.equal(rs[0], rs[1])
    s0, s1 = envs[0].shard.host_state(), envs[1].shard.host_state()
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k])


@pytest.mark.parametrize("tpw", [1, 2, 4, 8])
@pytest.mark.parametrize("mode", ["random", "buffer"])
def test_pipelined_step_bit_identical(tpw, mode):
    """k_step_pipe (MDR_OPT_STEP_TPW tiles per wave, next tile's loads issued before this tile's math) ==
    k_step_t bit for bit: ragged shard (odd size, partial last tile), fused random actions with
    lookahead and buffer actions, per-step API and graph rollouts."""
    import torch

    import golden_util as gu
    from mdr_amd.environment import Environment

    n = 100_003
    props = gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    envs = []
    for t in (0, tpw):
        e = Environment(props, rng=random.Random(2), population="synthetic", seed=3)
        e.shard.set_option("step_tpw", t)
        envs.append(e)
    g = torch.Generator(device="cuda").manual_seed(11)
    for t in range(25):
        if mode == "random":
            rs = [e.step_tensor(None, action_mode="random", lookahead="random").clone() for e in envs]
        else:
            a = (torch.rand(n, device="cuda", generator=g) < 0.5).to(torch.uint8)
            rs = [e.step_tensor(a, action_mode="buffer").clone() for e in envs]
        assert torch.equal(rs[0], rs[1]), f"tick {t}"
        assert float(envs[0].shard.p_dev.item()) == float(envs[1].shard.p_dev.item())
    acts = (torch.rand((30, n), device="cuda", generator=g) < 0.5).to(torch.uint8) if mode == "buffer" else None
    rr = [e.rollout(30, actions=acts, action_mode=mode) for e in envs]
    assert torch.equal(rr[0], rr[1])
    s0, s1 = envs[0].shard.host_state(), envs[1].shard.host_state()
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k])


@pytest.mark.parametrize("tpw", [0, 4])
def test_fast_division_guard_fallback(tpw):
    """Out-of-range parameters (Ua = 1e-9 < 2^-20) or temperatures route the tile to the plain
    `/` operator: results stay bit-identical to the reference-order kernel (k_step_t and
    k_step_pipe)."""
    import torch

    import golden_util as gu
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 5000,
                                     "power_grid_prop.signal_properties.mode": "flat"})
    envs = []
    for fast in (0, 1):
        e = Environment(props, rng=random.Random(2), population="synthetic", seed=3)
        e.shard.set_option("fastdiv", fast)
        e.shard.set_option("step_tpw", tpw if fast else 0)
        e.shard.ua[17] = 1e-9
        e.shard.t_air[4000] = 3.0e6
        e.shard.params_changed()
        envs.append(e)
    for t in range(10):
        rs = [e.step_tensor(None, action_mode="random", lookahead="random").clone() for e in envs]
        assert torch.equal(rs[0], rs[1])
    s0, s1 = envs[0].shard.host_state(), envs[1].shard.host_state()
    np.testing.assert_array_equal(s0["T"], s1["T"])
    np.testing.assert_array_equal(s0["Tm"], s1["Tm"])
