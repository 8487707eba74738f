"""Debug: the wide golden case (closed groups, every optional feature) in the fp16-split fp32 form,
per-house probability errors against torch fp32, the actor status, and the same rows re-run in the
three-way bf16 form."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

import golden_util as gu
from mdr_amd.actor import DeviceActor, make_actor
from mdr_amd.environment import Environment

case = sys.argv[1] if len(sys.argv) > 1 else "n30_maxerr_groups_hvacmsg"
d, meta = gu.traj(case)
props = gu.props_from_overrides(meta["overrides"])
for form in ("f16_split", "bf16_split3"):
    env = Environment(props, rng=random.Random(meta["seed"]))
    for _ in range(meta["resets"] - 1):
        env.reset(return_obs=False)
    F = env.obs_spec().n_feat
    actor = make_actor(F, 2, [100, 100], seed=1).to("cuda")
    da = DeviceActor(env, actor, precision="fp32", fp32_form=form)
    N = env.n_local
    probs = torch.empty((N, 2), dtype=torch.float32, device="cuda")
    obs = torch.empty((N, F), dtype=torch.float32, device="cuda")
    da.select_actions(probs=probs, obs_out=obs, count_next=False)
    with torch.no_grad():
        tp = actor(obs).cpu().numpy()
    p = probs.cpu().numpy()
    err = np.abs(p - tp).max(1)
    print(form, "F", F, "status", da.status(), "max err", err.max(), "bad houses", np.nonzero(err > 1e-5)[0][:40])
    print("  obs absmax per feature", np.round(obs.abs().amax(0).cpu().numpy(), 3).tolist())
    print("  p[:4]", p[:4].tolist(), "tp[:4]", tp[:4].tolist())
