"""A/B of the greedy select's launch forms on config C3 (1M houses, bench.py's population): HIP
events around mdr_greedy_rollout calls of 100 ticks, alternating MDR_OPT_GQ_BAND 1 / 0 on one
context (the drivers are computed before each call's first event).  Prints per-tick medians and the
band's skip / miss counts.  Usage: python tools/greedy_ab.py [reps] [step_tpw]"""
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "marl-demandresponse_amd"))

import torch  # noqa: E402

from bench import env_props  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n, K = 1 << 20, 100
    env = Environment(env_props(n), device="cuda:0", rng=random.Random(4), population="synthetic", seed=1234)
    sh = env.shard
    if len(sys.argv) > 2:
        sh.set_option("step_tpw", int(sys.argv[2]))
    act = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rew = torch.empty(n, dtype=torch.float64, device="cuda:0")
    env.greedy_rollout(150, actions=act, rewards=rew)  # warm: keys, map, band in steady state
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {0: [], 1: []}
    for r in range(reps):
        for band in (1, 0):
            sh.set_option("gq_band", band)
            ticks = env.driver_window(K)
            b0 = sh.greedy_band()
            torch.cuda.synchronize()
            ev0.record()
            sh.greedy_rollout(ticks, act, 0, rew, 0)
            ev1.record()
            torch.cuda.synchronize()
            us = ev0.elapsed_time(ev1) * 1000.0 / K
            b1 = sh.greedy_band()
            res[band].append(us)
            print(f"rep {r} band {band}: {us:.2f} us/tick, skips {b1['skips'] - b0['skips']} of {K}", flush=True)
    for band in (1, 0):
        print(f"band {band}: median {statistics.median(res[band]):.2f} us/tick over {reps} x {K} ticks")


if __name__ == "__main__":
    main()
