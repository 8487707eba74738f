"""The band's miss path priced: greedy calls at budgets drawn at random across the cluster's power
(every call misses the predicted band), band on / off alternating, each followed by a GQ step; run
under rocprofv3 --kernel-trace and compare the greedy kernels' summed durations per call."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "marl-demandresponse_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import env_props  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402

n = 1 << 20
props = env_props(n)
env = Environment(props, device="cuda:0", rng=random.Random(4), population="synthetic", seed=1234)
sh = env.shard
prm = sh.host_params()
p_all = float(np.sum(np.array(env._cap_values, np.float64)[prm["cap_idx"]]) / props.cluster_prop.house_prop.hvac_prop.cop)
act = torch.empty(n, dtype=torch.uint8, device="cuda:0")
rs = np.random.RandomState(3)
env.greedy_rollout(20, actions=act)
for band in (1, 0, 1, 0):
    sh.set_option("gq_band", band)
    for _ in range(50):
        sh.greedy(p_all * float(rs.uniform(0.05, 0.95)), act)
        env.step_tensor(act, ctrl="greedy_keys")
torch.cuda.synchronize()
print("band", sh.greedy_band())
