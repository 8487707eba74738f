"""Where does the time of a short timed region go?  (host drivers / C launch / sync / device)

    python tools/overhead.py [--houses 1048576] [--ticks 20] [--idle-ms 0,50]

Replays the bench's timed region (driver_window + graph rollout + synchronize) several times and
prints per-phase host microseconds and the launch-stream event window, right after the previous
iteration and after an idle gap (GPU clock ramp / queue wake-up effects)."""
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
    ap.add_argument("--idle-ms", default="0,50")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    from bench import env_props
    from mdr_amd.environment import Environment

    dev = torch.device("cuda", 0)
    n, T = a.houses, a.ticks
    env = Environment(env_props(n), device=dev, rng=random.Random(4), population="synthetic", seed=1234)
    sh = env.shard
    rew = torch.empty((T, n), dtype=torch.float64, device=dev)
    env.rollout(T, rewards=rew)  # capture
    env.rollout(T, rewards=rew)
    torch.cuda.synchronize()
    ls = env.rollout_stream()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    for idle in [float(x) for x in a.idle_ms.split(",")]:
        for r in range(a.reps):
            if idle:
                time.sleep(idle / 1e3)
            t0 = time.perf_counter()
            e0.record(ls)
            ticks = env.driver_window(T)
            t1 = time.perf_counter()
            sh.rollout(ticks, None, 0, 1, rew, n, True)
            t2 = time.perf_counter()
            e1.record(ls)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            print(f"idle {idle:5.0f} ms rep {r}: drivers {1e6 * (t1 - t0):7.1f} us  C rollout call "
                  f"{1e6 * (t2 - t1):7.1f} us  sync wait {1e6 * (t3 - t2):7.1f} us  wall {1e6 * (t3 - t0):7.1f} us  "
                  f"event window {1e3 * e0.elapsed_time(e1):7.1f} us", flush=True)
    # the bench's own call: Environment.rollout (drivers + C call), one timed region per rep
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(ls)
        env.rollout(T, rewards=rew)
        t1 = time.perf_counter()
        e1.record(ls)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"env.rollout rep {r}: call {1e6 * (t1 - t0):7.1f} us  wall {1e6 * (t2 - t0):7.1f} us  "
              f"event window {1e3 * e0.elapsed_time(e1):7.1f} us", flush=True)
    # the launch-first sequence of Environment.rollout, phase by phase
    from mdr_amd import _lib as L
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(ls)
        sh.rollout_launch(T, env._tick, None, 0, L.ACT_RANDOM, rew, n)
        t1 = time.perf_counter()
        ticks = env.driver_window(T)
        t2 = time.perf_counter()
        sh.rollout(ticks, None, 0, L.ACT_RANDOM, rew, n, True)
        t3 = time.perf_counter()
        env._P_dev_valid = True
        env.finish_grid_step()
        t4 = time.perf_counter()
        e1.record(ls)
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        print(f"launch-first rep {r}: launch {1e6 * (t1 - t0):6.1f} us  drivers {1e6 * (t2 - t1):6.1f} us  "
              f"post {1e6 * (t3 - t2):6.1f} us  grid {1e6 * (t4 - t3):6.1f} us  sync {1e6 * (t5 - t4):6.1f} us  "
              f"wall {1e6 * (t5 - t0):6.1f} us  event {1e3 * e0.elapsed_time(e1):6.1f} us  "
              f"launched {sh.rollout_launched()}", flush=True)
    # device-only replay of the same graph (no host drivers): the floor of the timed region
    for r in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(ls)
        sh.rollout(ticks, None, 0, 1, rew, n, True)
        e1.record(ls)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print(f"graph only rep {r}: wall {1e6 * (t1 - t0):7.1f} us  event {1e3 * e0.elapsed_time(e1):7.1f} us")


if __name__ == "__main__":
    main()
