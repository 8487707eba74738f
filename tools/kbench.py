"""Kernel A/B microbenchmark for k_step (one process, interleaved rounds; cdna guide §5.4 r24).

    python tools/kbench.py [--houses 1048576,4194304] [--launches 200] [--rounds 5]
Prints per-launch microseconds and algorithmic GB/s (99 B/house-step) per variant, plus the
memory-floor probe (same loads/stores, no arithmetic).
"""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", default="1048576,4194304,16777216")
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="hpt2,fast2,fcoef2,probe")
    a = ap.parse_args()
    import torch

    from bench import env_props
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    res = {}
    for n in [int(x) for x in a.houses.split(",")]:
        envs = {}
        for v in a.variants.split(","):
            os.environ["MDR_HPT"] = "1" if v.endswith("1") else "2"
            os.environ["MDR_VARIANT"] = "coef" if "coef" in v else "raw"
            os.environ["MDR_FASTDIV"] = "1" if v.startswith("f") else "0"
            os.environ["MDR_GRID_OVERSUB"] = v.split("g")[-1] if "g" in v[4:] else "1"
            os.environ["MDR_TPW"] = v.split("t")[-1] if "t" in v[4:] else "0"  # fast2t4: k_step_pipe, 4 tiles/wave
            envs[v] = Environment(env_props(n), device="cuda:0", rng=random.Random(1),
                                  population="synthetic", seed=5)
            rews = torch.empty(n, dtype=torch.float64, device="cuda:0")
            # one driver window replayed every round: the events time the graph alone (no host drivers)
            envs[v]._kb_ticks = envs[v].driver_window(a.launches)
            sh = envs[v].shard
            sh.rollout(envs[v]._kb_ticks, None, 0, L.ACT_RANDOM, rews, 0, True)  # captures the graph
            envs[v]._kb_rew = rews
        torch.cuda.synchronize()
        for r in range(a.rounds):
            for v, env in envs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                sh = env.shard
                if v == "probe":
                    e0.record()
                    for _ in range(a.launches):
                        L.check(sh.lib.mdr_probe_stream(sh.ctx, L.ptr(sh.reward), sh.stream()))
                    e1.record()
                else:
                    torch.cuda.synchronize()
                    ls = sh.launch_stream(True)
                    sh.rollout(env._kb_ticks, None, 0, L.ACT_RANDOM, env._kb_rew, 0, True)  # stage ticks
                    e0.record(ls)
                    sh.rollout(env._kb_ticks, None, 0, L.ACT_RANDOM, env._kb_rew, 0, True)
                    e1.record(ls)
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.launches
                res.setdefault((n, v), []).append(us)
        for v in envs:
            ts = sorted(res[(n, v)])
            med = ts[len(ts) // 2]
            print(f"n={n:>9} {v:>6}: {med:8.2f} us/launch (min {ts[0]:.2f})  "
                  f"{99 * n / med / 1e3:8.1f} GB/s algorithmic  {n / med * 1e6:.3e} house-steps/s", flush=True)
        del envs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
