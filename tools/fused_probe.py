"""Phase stamps of k_window_fused (mdr_fused_stamps): per block the 100 MHz clock at entry, after its
count flush, after the grid-wide wait, at the end of its thermal loop; printed as percentiles over
blocks relative to the first block's entry, for rollout(K) calls at N houses (fused on), next to
the wall time of the same calls with the count + step kernel pair."""
import argparse
import ctypes as C
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as gu  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--houses", type=int, default=1 << 20)
ap.add_argument("--ticks", type=int, default=20)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
props = gu.props_from_overrides({"cluster_prop.nb_agents": a.houses,
                                 "power_grid_prop.signal_properties.mode": "sinusoidals"})
env = Environment(props, rng=random.Random(4), population="synthetic", seed=1234)
sh = env.shard
rew = torch.empty((a.ticks, a.houses), dtype=torch.float64, device="cuda")
buf = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
for fused in (1, 0):
    sh.set_option("window_fused", fused)
    for _ in range(5):
        env.rollout(a.ticks, rewards=rew)
    torch.cuda.synchronize()
    walls = []
    for r in range(a.reps):
        last = r == a.reps - 1
        if fused and last:
            sh.lib.mdr_fused_stamps(sh.ctx, C.c_void_p(buf.data_ptr()), buf.numel())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.rollout(a.ticks, rewards=rew)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        if fused and last:
            sh.lib.mdr_fused_stamps(sh.ctx, None, 0)
    print(f"fused={fused}: rollout({a.ticks}) at {a.houses:,} houses: wall median {1e6 * np.median(walls):.1f} us "
          f"min {1e6 * min(walls):.1f}", flush=True)
    if fused:
        st = buf.cpu().numpy().astype(np.int64)
        nb = int(np.count_nonzero(st[0::8]))
        st = st[:8 * nb].reshape(nb, 8)
        nc = min(256, nb)  # count blocks: one per CU (mdr_capi.hip launch_fused)
        base = st[:, 0].min()
        rel = (st - base) / 100.0  # us
        def show(name, v):
            q = np.percentile(v, [0, 50, 90, 100])
            print(f"  {name:34s} min {q[0]:6.1f} p50 {q[1]:6.1f} p90 {q[2]:6.1f} max {q[3]:6.1f} us")
        c, t = rel[:nc], rel[nc:]
        show("count blocks: entry", c[:, 0])
        show("count blocks: flushed", c[:, 1])
        show("count blocks: done (last = published)", c[:, 2])
        show("thermal blocks: entry", t[:, 0])
        show("thermal blocks: coefficients", t[:, 1])
        show("thermal blocks: flag seen", t[:, 2])
        show("thermal blocks: end", t[:, 3])
        print(f"  {nc} count + {nb - nc} thermal blocks; thermal blocks that waited for the flag: "
              f"{int(np.sum(t[:, 2] - t[:, 1] > 0.5))}", flush=True)
