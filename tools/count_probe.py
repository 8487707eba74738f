"""k_count_window alone (the first window's FSM count of a rollout), for rocprofv3 --kernel-trace:

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/count_probe.py
    python3 tools/count_probe.py --analyze OUT/run_kernel_trace.csv

Launches REPS counts for each (mode, ticks) pair in a fixed order (mdr_rollout_begin; every
launch discards the previous one), synchronising between groups; --analyze prints the average
kernel duration per group from the trace, in the same order."""
import argparse
import csv
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]
TICKS = [1, 4, 8, 16, 20, 32]
MODES = ["random", "always_on"]
REPS = 20


def groups():
    ticks = [int(x) for x in os.environ.get("CP_TICKS", ",".join(map(str, TICKS))).split(",")]
    modes = os.environ.get("CP_MODES", ",".join(MODES)).split(",")
    return [(m, t) for m in modes for t in ticks]


def run(houses):
    import torch

    from bench import env_props
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    env = Environment(env_props(houses), device="cuda:0", rng=random.Random(1), population="synthetic", seed=5)
    sh = env.shard
    modes = {"random": L.ACT_RANDOM, "always_on": L.ACT_ALWAYS_ON}
    for m, t in groups():
        for _ in range(REPS):
            sh.rollout_begin(t, 0, None, 0, modes[m])
        torch.cuda.synchronize()
    print("done", len(groups()) * REPS, "counts")


def analyze(path):
    rows = [r for r in csv.DictReader(open(path)) if "k_count_window" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    for i, (m, t) in enumerate(groups()):
        g = sorted(d[i * REPS:(i + 1) * REPS])[2:-2]  # trimmed
        if g:
            print(f"{m:10s} ticks {t:3d}: {sum(g) / len(g):7.2f} us (min {g[0]:.2f})")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--analyze")
    a = ap.parse_args()
    analyze(a.analyze) if a.analyze else run(a.houses)
