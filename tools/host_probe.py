"""Host-side cost of one short rollout call (the driver's --steps 20 bench shape), piece by piece:
Environment.rollout's Python, mdr_rollout_begin, the drivers, the launching mdr_rollout call.
Each piece is timed over many calls with the device drained in between (so the launch queue never
fills), min and median in microseconds.

    python tools/host_probe.py [--houses 1048576] [--ticks 20] [--reps 300]
"""
import argparse
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--idle", default="none", choices=["none", "spin", "sleep"],
                    help="before each timed call: nothing, a 3 ms busy loop (bench.py's host spin), a 3 ms sleep")
    a = ap.parse_args()
    import torch

    import bench
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    env = Environment(bench.env_props(a.houses), device="cuda:0", rng=random.Random(4), population="synthetic",
                      seed=1234)
    sh = env.shard
    n = a.ticks
    rew = torch.empty((n, env.n_local), dtype=torch.float64, device="cuda:0")
    for _ in range(20):
        env.rollout(n, action_mode="random", rewards=rew)
    torch.cuda.synchronize()
    res = {k: [] for k in ("rollout (whole call)", "rollout_begin", "driver_window", "shard.rollout", "sync",
                           "python before the fused C call", "fused C call", "python after the fused C call")}
    # the fused path (Environment.rollout -> _host.rollout1): stamp the C call's entry and exit
    import mdr_amd.environment as E

    host = E._host
    stamps = []

    class _Shim:
        drivers = staticmethod(host.drivers)

        @staticmethod
        def rollout1(*args):
            stamps.append(time.perf_counter())
            r = host.rollout1(*args)
            stamps.append(time.perf_counter())
            return r

    E._host = _Shim
    def idle():
        if a.idle == "spin":
            t = time.perf_counter()
            while time.perf_counter() - t < 3e-3:
                pass
        elif a.idle == "sleep":
            time.sleep(3e-3)

    for _ in range(a.reps):
        torch.cuda.synchronize()
        idle()
        t0 = time.perf_counter()
        stamps.clear()
        env.rollout(n, action_mode="random", rewards=rew)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res["rollout (whole call)"].append(t1 - t0)
        res["sync"].append(t2 - t1)
        if len(stamps) == 2:
            res["python before the fused C call"].append(stamps[0] - t0)
            res["fused C call"].append(stamps[1] - stamps[0])
            res["python after the fused C call"].append(t1 - stamps[1])
        # the pieces, as Environment.rollout issues them
        torch.cuda.synchronize()
        idle()
        t0 = time.perf_counter()
        sh.rollout_begin(n, env._tick, None, 0, L.ACT_RANDOM)
        t1 = time.perf_counter()
        ticks = env.driver_window(n)
        t2 = time.perf_counter()
        sh.rollout(ticks, None, 0, L.ACT_RANDOM, rew, env.n_local, False)
        t3 = time.perf_counter()
        env._P_dev_valid = True
        env.finish_grid_step()
        res["rollout_begin"].append(t1 - t0)
        res["driver_window"].append(t2 - t1)
        res["shard.rollout"].append(t3 - t2)
    torch.cuda.synchronize()
    for k, v in res.items():
        if not v:
            continue
        print(f"{k:>22s}: min {1e6 * min(v):7.1f} us  median {1e6 * statistics.median(v):7.1f} us")


if __name__ == "__main__":
    main()
