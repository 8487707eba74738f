"""The fused obs + actor kernel alone (k_actor via DeviceActor.select_actions, no step), HIP events
around K launches: the per-launch time and achieved TFLOP/s on the algorithmic FLOPs; the program
rocprofv3 --pmc passes profile (tools/pmc_actor.sh).

    python tools/actor_kbench.py [--houses 1048576] [--precision bf16x3] [--reps 20] [--fp32-form f16_split]
"""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--precision", default="bf16x3")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--fp32-form", default="f16_split", choices=["f16_split", "bf16_split3"])
    a = ap.parse_args()
    import torch

    import bench
    from mdr_amd.actor import DeviceActor, make_actor
    from mdr_amd.environment import Environment

    env = Environment(bench.env_props(a.houses), device="cuda:0", rng=random.Random(4), population="synthetic",
                      seed=1234)
    actor = make_actor(env.obs_spec().n_feat, 2, [100, 100], seed=1)
    da = DeviceActor(env, actor, precision=a.precision, fp32_form=a.fp32_form)
    n = env.n_local
    act = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    prob = torch.empty(n, dtype=torch.float32, device="cuda:0")
    for _ in range(3):
        da.select_actions(action=act, prob=prob, count_next=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        da.select_actions(action=act, prob=prob, count_next=False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    flops = 2 * sum(l.in_features * l.out_features for l in actor.fc) * n
    st = da.status()
    print(f"houses={n} precision={a.precision} kernel_prec={st['kernel_prec']} range_faults={st['range_faults']} exact_tiles={st['exact']}: k_actor {us:.1f} us/launch, {flops / us / 1e6:.1f} TFLOP/s "
          f"algorithmic ({flops / us / 1e6 / bench.BF16_PEAK_TFS:.3f} of dense bf16 peak)", flush=True)


if __name__ == "__main__":
    main()
