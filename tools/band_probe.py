"""Probe of the greedy select's predicted band on bench.py's C3 loop (1M houses): per tick, the
band the step epilogue counted (GqSel.band_base before the call), the crossing superbin the call
found, and whether k_gq_binsc skipped the bins pass.  Usage: python tools/band_probe.py [ticks]"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "marl-demandresponse_amd"))

import torch  # noqa: E402

from bench import env_props  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402


def main():
    ticks = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    n = 1 << 20
    env = Environment(env_props(n), device="cuda:0", rng=random.Random(4), population="synthetic", seed=1234)
    sh = env.shard
    act = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rows = []
    kband = sh.greedy_band()["band_width"]
    for t in range(ticks):
        b0 = sh.greedy_band()
        env.greedy_actions(out=act)
        b1 = sh.greedy_band()
        st = sh.greedy_state()
        env.step_tensor(act, ctrl="greedy_keys")
        rows.append((t, b0["band_base"], st["sb"], st["bstar"], b1["skips"] - b0["skips"], st["window_last"]))
        print("t=%3d band=[%3d,%3d) sb=%3d bstar=%5d skip=%d window=%d" % (t, rows[-1][1], rows[-1][1] + kband,
                                                                          *rows[-1][2:]), flush=True)
    d = [r[2] - r[1] for r in rows[1:]]
    print("sb - band_base: min %d max %d mean %.2f; skips %d of %d" % (min(d), max(d), sum(d) / len(d),
                                                                     sum(r[4] for r in rows), len(rows)))


if __name__ == "__main__":
    main()
