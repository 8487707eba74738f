"""Per-phase shader-cycle profile of the fused actor kernel (mdr_actor_profile) at bench scale.

    python tools/actor_profile.py [--houses N] [--precision bf16x3|bf16]
"""
import argparse
import ctypes as C
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]

PHASES = ["weights+barrier", "obs build", "prefetch+obs_out", "layer 1", "layer 2", "out+softmax", "-", "tiles"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--precision", default="bf16x3")
    a = ap.parse_args()
    import torch

    import bench
    from mdr_amd import _lib as L
    from mdr_amd.actor import DeviceActor, make_actor
    from mdr_amd.environment import Environment

    env = Environment(bench.env_props(a.houses), device="cuda:0", rng=random.Random(4), population="synthetic",
                      seed=1234)
    da = DeviceActor(env, make_actor(env.obs_spec().n_feat, 2, [100, 100], seed=1), precision=a.precision)
    spec, sc, keep = env.bound_obs_spec()
    sh = env.shard
    out = (C.c_double * 8)()
    for _ in range(3):
        L.check(sh.lib.mdr_actor_profile(sh.ctx, C.byref(spec), C.byref(sc), 0, out, sh.stream()), "profile")
    tot = sum(out[k] for k in range(7))
    print(f"houses={a.houses} precision={a.precision} tiles/wave={out[7]:.1f} total={tot:.0f} cycles "
          f"({tot / 2.4e3:.1f} us at 2.4 GHz)")
    for k in range(7):
        print(f"  {PHASES[k]:>24s}: {out[k]:10.0f} cycles  {100 * out[k] / max(tot, 1):5.1f} %  "
              f"per tile {out[k] / max(out[7], 1):8.0f}")


if __name__ == "__main__":
    main()
