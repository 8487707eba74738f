"""Debug probe: the chained actor's rollout graph vs the select_actions / step_tensor loop."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import golden_util as gu  # noqa: E402
from mdr_amd.actor import DeviceActor  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402


def env(n, seed):
    return Environment(gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                                "power_grid_prop.signal_properties.mode": "sinusoidals"}),
                       rng=random.Random(seed))


for layers, graph in (((64, 64, 64), True), ((64, 64, 64), False), ((100, 100), True)):
    n, T = 2049, 6
    ea, eb = env(n, 8), env(n, 8)
    m = ea.obs_tensor().abs().amax(0).double().cpu().numpy()
    actor = gu.calibrated_actor(ea.obs_spec().n_feat, m, seed=2, layers=layers).to("cuda")
    da, db = DeviceActor(ea, actor), DeviceActor(eb, actor)
    rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
    acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    for rep in range(3):
        da.rollout(T, rewards=rew, actions=acts, use_graph=graph)
        bad = []
        for t in range(T):
            a, p = db.select_actions(count_next=True)
            r = eb.step_tensor(a)
            if not (torch.equal(a, acts[t]) and torch.equal(r, rew[t])):
                bad.append((t, int((a != acts[t]).sum()), float(rew[t][0]), float(r[0])))
        print(layers, "graph" if graph else "direct", "rep", rep, "fused", da.fused(), "P", ea._cluster_power(),
              eb._cluster_power(), "bad", bad, flush=True)
