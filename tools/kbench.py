"""Kernel A/B microbenchmark for the step kernels (one process, interleaved rounds; cdna guide §5.4).

    python tools/kbench.py [--houses 1048576,4194304] [--ticks 128] [--rounds 5] [--variants w32,w0,probe]

Variants: wK[e] = temporally blocked rollout, K ticks per k_step_window launch (affine per-window
thermal transition; e = the exact per-tick expression, MDR_OPT_WINDOW_THERMAL); w0 = one launch per
tick (k_step_pipe); probe =
the memory-floor probe of the one-tick kernel (same loads/stores, no arithmetic).  Every tick's
reward row is kept ([ticks, n] float64), so reward writes really go to HBM.  Prints per-tick
microseconds, house-steps/s and algorithmic GB/s (window: SURVEY §8(d) field sizes, state and
parameters once per window + 8 B reward per tick; one-tick: 99 B/house-step).
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
    ap.add_argument("--ticks", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="w32,w32e,w16,w0,probe")
    a = ap.parse_args()
    import torch

    from bench import BYTES_PER_HOUSE_STEP, env_props, window_bytes
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    res = {}
    for n in [int(x) for x in a.houses.split(",")]:
        envs = {}
        for v in a.variants.split(","):
            env = Environment(env_props(n), device="cuda:0", rng=random.Random(1), population="synthetic", seed=5)
            sh = env.shard
            if v.startswith("w"):
                sh.set_rollout_window(int(v[1:].rstrip("e")))
                sh.set_option("window_thermal", L.THERMAL_EXACT if v.endswith("e") else L.THERMAL_AFFINE)
            env._kb_rew = torch.empty((a.ticks, n), dtype=torch.float64, device="cuda:0")
            # one driver window replayed every round: the events time the graph alone (no host drivers)
            env._kb_ticks = env.driver_window(a.ticks)
            if v != "probe":
                sh.rollout(env._kb_ticks, None, 0, L.ACT_RANDOM, env._kb_rew, n, True)  # captures the graph
            envs[v] = env
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()  # torch creates the HIP events lazily on the first record(): not inside a timing
        e1.record()
        for r in range(a.rounds):
            for v, env in envs.items():
                sh = env.shard
                if v == "probe":
                    e0.record()
                    for t in range(a.ticks):
                        L.check(sh.lib.mdr_probe_stream(sh.ctx, L.ptr(env._kb_rew[t]), sh.stream()))
                    e1.record()
                else:
                    torch.cuda.synchronize()
                    ls = sh.launch_stream()
                    e0.record(ls)
                    sh.rollout(env._kb_ticks, None, 0, L.ACT_RANDOM, env._kb_rew, n, True)
                    e1.record(ls)
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.ticks
                res.setdefault((n, v), []).append(us)
        for v in envs:
            ts = sorted(res[(n, v)])
            med = ts[len(ts) // 2]
            if v.startswith("w") and int(v[1:].rstrip("e")) > 0:
                k = int(v[1:].rstrip("e"))
                launches = -(-a.ticks // k)
                kk = a.ticks // launches
                gbs = window_bytes(n, kk, "random") / (med * kk) / 1e3
            else:
                gbs = BYTES_PER_HOUSE_STEP * n / med / 1e3
            print(f"n={n:>9} {v:>6}: {med:8.2f} us/tick (min {ts[0]:.2f})  {gbs:8.1f} GB/s algorithmic  "
                  f"{n / med * 1e6:.3e} house-steps/s", flush=True)
        del envs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
