"""Bisect probe: which node of the chained actor's captured rollout leaves non-zero values in the
count slab that only the graph's leading memset touches (slab 1 after a 1-tick rollout)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import golden_util as gu  # noqa: E402
from mdr_amd.actor import DeviceActor  # noqa: E402
from mdr_amd.distributed import device_view  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402

n, T = 2049, 1
e = Environment(gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                         "power_grid_prop.signal_properties.mode": "sinusoidals"}),
                rng=random.Random(8))
m = e.obs_tensor().abs().amax(0).double().cpu().numpy()
layers = tuple(int(x) for x in os.environ.get("LAYERS", "64,64,64").split(","))
actor = gu.calibrated_actor(e.obs_spec().n_feat, m, seed=2, layers=layers).to("cuda")
da = DeviceActor(e, actor)
rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
res = []
for rep in range(4):
    da.rollout(T, rewards=rew, actions=acts, use_graph=True)
    ptr, ln = e.shard.counts_buffer()  # ring 1 after T = 1: slab 1, written only by the memset
    torch.cuda.synchronize()
    v = device_view(ptr, ln, "<i8", "cuda").clone().cpu()
    res.append(int((v != 0).sum()))
print("skip", os.environ.get("MDR_DBG_CHAIN_SKIP", "0"), "zero_kernel", int("MDR_DBG_ZERO_KERNEL" in os.environ),
      "layers", layers, "fused", da.fused(), "nonzero entries of slab 1 per rep", res, flush=True)
