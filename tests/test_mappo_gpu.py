"""MA-PPO update on device (mdr_amd.mappo.DeviceMAPPO) against one reference MAPPO.update
(tests/golden/mappo.npz, made by make_golden.gen_mappo at N = 2 where the reference critic runs):
identical initial weights (same torch.manual_seed init order), the same minibatch order (global
CPU generator), and final weights within float32 accumulation-order tolerance (GPU matmuls)."""
import json
import random

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu


def test_mappo_update_matches_reference():
    import torch

    from mdr_amd.environment import Environment
    from mdr_amd.mappo import DeviceMAPPO, MAPPOConfig

    z = gu.load("mappo.npz")
    meta = json.loads(bytes(z["meta_json"]).decode())
    props = gu.props_from_overrides({"cluster_prop.nb_agents": 2,
                                     "power_grid_prop.signal_properties.mode": "flat"})
    env = Environment(props, rng=random.Random(1))
    agent = DeviceMAPPO(env, MAPPOConfig(batch_size=meta["batch_size"], ppo_update_time=meta["ppo_update_time"]),
                        seed=meta["seed"])
    assert agent.num_state == meta["num_state"]
    for net, tag in ((agent.actor_net, "actor"), (agent.critic_net, "critic")):
        for k, v in net.state_dict().items():
            np.testing.assert_array_equal(v.cpu().numpy(), z[f"init_{tag}_{k}"], err_msg=f"init {tag} {k}")
    dev = env.shard.device
    S = torch.from_numpy(z["states"]).to(dev)
    for t in range(meta["T"]):
        agent.last_actions = torch.from_numpy(z["actions"][t].astype(np.uint8)).to(dev)
        agent.last_probs = torch.from_numpy(z["probs"][t]).to(dev)
        agent.store_transition(S[t], S[t + 1], torch.from_numpy(z["rewards"][t]).to(dev), bool(z["done"][t]))
    assert len(agent) == 2 * meta["T"]
    torch.manual_seed(meta["update_seed"])
    assert agent.update(meta["T"])
    assert agent.training_step == meta["training_steps"]
    for net, tag in ((agent.actor_net, "actor"), (agent.critic_net, "critic")):
        for k, v in net.state_dict().items():
            np.testing.assert_allclose(v.cpu().numpy(), z[f"final_{tag}_{k}"], rtol=2e-3, atol=2e-4,
                                       err_msg=f"final {tag} {k}")


@pytest.mark.parametrize("sampler", ["reference", "device"])
def test_training_loop_runs_on_device(sampler):
    """TrainingManager-style loop (training_manager.py:183-263) at 4,099 houses: select_actions ->
    step -> store_transition -> update every epoch; the update runs and the policy moves (minibatch
    permutations from the CPU generator, as the reference, or from the device generator)."""
    import torch

    from mdr_amd.environment import Environment
    from mdr_amd.mappo import DeviceMAPPO, MAPPOConfig

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 4099,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(2), population="synthetic", seed=3)
    agent = DeviceMAPPO(env, MAPPOConfig(batch_size=4096, ppo_update_time=2), sampler=sampler)
    w0 = agent.actor_net.fc[0].weight.detach().clone()
    obs = env.obs_tensor().clone()
    for t in range(6):
        a = agent.select_actions()
        r = env.step_tensor(a).clone()
        nxt = env.obs_tensor().clone()
        agent.store_transition(obs, nxt, r, done=(t == 5))
        obs = nxt
    assert agent.update(5)
    assert len(agent) == 0 and not torch.equal(w0, agent.actor_net.fc[0].weight.detach())
    assert torch.isfinite(agent.actor_net.fc[0].weight).all()
