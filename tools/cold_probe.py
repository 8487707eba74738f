"""Host phases of ONE short rollout call after an idle host spin (the bench's timed region shape),
per launch policy: launch-first direct (default), launch-first graph (MDR_LF_GRAPH=1 in the
environment of this process), begin + kernel-argument drivers (--kernarg).

    python tools/cold_probe.py [--ticks 20] [--reps 8] [--spin-ms 3] [--kernarg]"""
import argparse
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--spin-ms", type=float, default=3.0)
    ap.add_argument("--kernarg", action="store_true")
    a = ap.parse_args()
    import torch

    from bench import env_props
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    dev = torch.device("cuda", 0)
    n, T = a.houses, a.ticks
    env = Environment(env_props(n), device=dev, rng=random.Random(4), population="synthetic", seed=1234)
    sh = env.shard
    rew = torch.empty((T, n), dtype=torch.float64, device=dev)
    for _ in range(4):
        env.rollout(T, rewards=rew, use_graph=not a.kernarg)
    torch.cuda.synchronize()
    tag = "kernarg" if a.kernarg else ("lf-graph" if os.environ.get("MDR_LF_GRAPH") else "lf-direct")
    for r in range(a.reps):
        torch.cuda.synchronize()
        ts = time.perf_counter()
        while time.perf_counter() - ts < a.spin_ms * 1e-3:
            pass
        t0 = time.perf_counter()
        if a.kernarg:
            sh.rollout_begin(T, env._tick, None, 0, L.ACT_RANDOM)
        else:
            sh.rollout_launch(T, env._tick, None, 0, L.ACT_RANDOM, rew, n)
        t1 = time.perf_counter()
        ticks = env.driver_window(T)
        t2 = time.perf_counter()
        sh.rollout(ticks, None, 0, L.ACT_RANDOM, rew, n, not a.kernarg)
        t3 = time.perf_counter()
        env._P_dev_valid = True
        env.finish_grid_step()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"{tag:9s} rep {r}: launch/begin {1e6 * (t1 - t0):6.1f}  drivers {1e6 * (t2 - t1):6.1f}  "
              f"C call {1e6 * (t3 - t2):6.1f}  sync {1e6 * (t4 - t3):6.1f}  wall {1e6 * (t4 - t0):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
