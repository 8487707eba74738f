"""Captured graphs hold kernels only.

r04's captured rollouts began with a hipMemsetAsync node that left non-zero words in the count slabs
on every replay after the first; the library now zeroes with kernels and
capture_graph walks every captured graph before instantiating it, failing with MDR_EHIP on a
memset node.  These tests capture each rollout kind — the window rollout, the per-tick rollout
(window 0), the fused actor rollout and the actor layer chain — and assert through mdr_graph_info
that the guard walked each capture.  mdr_graph_memset_probe then captures a memset node in the
library's own context and reports its parameters against what was passed, and what its replays
leave in the slabs (printed: the record of whether ROCm's memset node itself misbehaves here).
"""
import random

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _env(n, extra=None, seed=5):
    from mdr_amd.environment import Environment

    ov = {"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "sinusoidals"}
    ov.update(extra or {})
    return Environment(gu.props_from_overrides(ov), rng=random.Random(seed), population="synthetic", seed=seed)


@pytest.mark.parametrize("kind", ["window", "per_tick", "actor_fused", "actor_chain"])
def test_every_capture_is_guarded(torch_gpu, kind):
    torch = torch_gpu
    n = 4099
    env = _env(n)
    g0 = env.shard.graph_info()
    if kind in ("window", "per_tick"):
        if kind == "per_tick":
            env.shard.set_rollout_window(0)
        for _ in range(3):
            env.rollout(12, action_mode="random", use_graph=True)
        gi = env.shard.graph_info()
        assert gi["rollout_graphs"] >= 1 and gi["rollout_launches"] >= g0["rollout_launches"] + 3, gi
    else:
        from mdr_amd.actor import DeviceActor

        layers = (100, 100) if kind == "actor_fused" else (64, 64, 64)
        m = env.obs_tensor().abs().amax(0).double().cpu().numpy()
        da = DeviceActor(env, gu.calibrated_actor(env.obs_spec().n_feat, m, seed=2, layers=layers).to("cuda"))
        assert da.fused() == (kind == "actor_fused")
        for _ in range(3):
            da.rollout(6)
        gi = env.shard.graph_info()
        assert gi["actor_graphs"] == 1 and gi["actor_launches"] == g0["actor_launches"] + 3, gi
    torch.cuda.synchronize()
    # every capture of this context went through the guard, and each graph had nodes to walk
    assert gi["guarded"] >= 1 and gi["guarded"] == gi["rollout_graphs"] + gi["actor_graphs"], gi
    assert gi["guarded_nodes"] >= gi["guarded"], gi


def test_memset_node_probe(torch_gpu):
    """A memset node captured in the library's context: the node's parameters equal what was
    passed (dst, value 0, 1-byte elements, the byte width, one row); the replays' slab contents are
    printed and recorded, and the kernel zeroing the library uses leaves no non-zero word."""
    torch = torch_gpu
    env = _env(2049)
    env.step_tensor(None, action_mode="random", lookahead="random")
    pr = env.shard.graph_memset_probe()
    print("memset probe:", pr)
    assert pr["memset_nodes"] == 1 and pr["dst_ok"] == 1, pr
    assert pr["value"] == 0 and pr["height"] == 1, pr
    assert pr["element_size"] * pr["width"] == pr["bytes"], pr
    assert pr["nonzero_kernel_zero"] == 0, pr
    # the context still steps correctly afterwards: the probe discarded the lookahead's counts (the
    # next step recounts them, phase 1), its twin keeps them
    env._counts_ready = 0
    twin = _env(2049)
    twin.step_tensor(None, action_mode="random", lookahead="random")
    ra = env.step_tensor(None, action_mode="random").clone()
    rb = twin.step_tensor(None, action_mode="random").clone()
    torch.cuda.synchronize()
    assert np.array_equal(ra.cpu().numpy(), rb.cpu().numpy())
