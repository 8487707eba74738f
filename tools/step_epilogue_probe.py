"""The GQ epilogue's price: the buffer-action step kernel at 1M houses with and without
ctrl='greedy_keys' (k_step_pipe<2, 0, 0, true / false>), 100 ticks each, for a rocprofv3 kernel trace."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "marl-demandresponse_amd"))

import torch  # noqa: E402

from bench import env_props  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402

n = 1 << 20
env = Environment(env_props(n), device="cuda:0", rng=random.Random(4), population="synthetic", seed=1234)
act = (torch.rand(n, device="cuda:0") < 0.3).to(torch.uint8)
for rep in range(2):
    for ctrl in (None, "greedy_keys"):
        for _ in range(100):
            env.step_tensor(act, ctrl=ctrl)
torch.cuda.synchronize()
print("done")
