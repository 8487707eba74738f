#!/usr/bin/env python
"""bench.py — vectorised env.step throughput (house-steps/s) on MI355X, with HBM roofline.

Workload (BASELINE.json metric "house-steps/s (env.step throughput) at 1M houses"): 1,048,576
houses per GPU (weak scaling: N_total = 1,048,576 x n_gpus), MARLconfig env_prop (dt = 4 s,
L = 40 s, individual_L2 rewards), sinusoidal regulation signal (perlin is parity-unpinned),
synthetic population drawn on device (Philox, the reference noise model), random actions from
the fused Philox controller (configs[1]'s controller; a tick is ONE fused HIP launch).  A step =
one env.step of every house: lockout FSM + RC thermal + cluster power + rewards, with the host
scalar drivers (outdoor temperature RNG, solar, signal) computed per tick inside the timed
region.  Ticks are issued as hipGraph-captured chunks (mdr_rollout); multi-GPU runs allreduce
the per-tick cluster-power counts with RCCL inside the loop (mdr_rollout_sharded).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--houses H] [--chunk C]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "marl-demandresponse_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "house-steps/s (env.step throughput) at 1M houses; % HBM roofline"
BYTES_PER_HOUSE_STEP = 99  # SURVEY §8(d) B_core: state r/w 42 + action 1 + params 48 + reward 8
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s
BF16_PEAK_TFS = 2516.6     # dense bf16 MFMA: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (no sparsity)



def step_kernel_name(n_loc: int, mode: str) -> str:
    """The k_step instantiation the library launches for this bench (launch_step_on in mdr_capi.hip)."""
    if any(k in os.environ for k in ("MDR_HPT", "MDR_VARIANT", "MDR_FASTDIV")):
        return "mdr::k_step (variant chosen by MDR_* env)"
    tpw = int(os.environ.get("MDR_TPW", 2 if n_loc <= 1572864 else 4))
    act = "RANDOM,RANDOM" if mode == "random" else "BUFFER,0"
    if tpw <= 0:
        return f"mdr::k_step_t<2,false,true,{act}>"
    tpw = 8 if tpw >= 8 else 4 if tpw >= 4 else 2 if tpw >= 2 else 1
    if mode != "random":
        tpw = 4 if tpw >= 4 else 2
    return f"mdr::k_step_pipe<{tpw},{act}>"

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--houses", type=int, default=1 << 20, help="houses per GPU")
    ap.add_argument("--chunk", type=int, default=100, help="ticks per graph-captured rollout call")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default="random", choices=["random", "buffer"])
    ap.add_argument("--workload", default="step", choices=["step", "actor"],
                    help="step: env.step with fused random actions (the BASELINE metric); actor: "
                         "config C5, MA-PPO actor select_actions fused with the obs, then env.step")
    ap.add_argument("--precision", default="bf16x3", choices=["bf16x3", "bf16"],
                    help="actor MFMA precision (--workload actor)")
    ap.add_argument("--comm", default="default", choices=["default", "none", "rccl", "torch"],
                    help="exchange for the sharded path (default: rccl when WORLD_SIZE > 1); "
                         "'rccl' at world 1 exercises the sharded C loop on one GPU")
    return ap.parse_args()


def env_props(n_total: int):
    from mdr_amd.config import EnvironmentProperties

    p = EnvironmentProperties.from_json(os.path.join(ROOT, "tests", "golden", "marl_env_prop.json"))
    p.cluster_prop.nb_agents = n_total
    p.power_grid_prop.signal_properties.mode = "sinusoidals"
    return p


def cpu_baseline(budget_s: float):
    """Oracle (oracle/env_np.py, NumPy fp64) on a bounded sample of the same workload."""
    import numpy as np

    from oracle import env_np as O

    n = 65536
    props = env_props(n)
    rs = np.random.RandomState(0)
    hp = props.cluster_prop.house_prop
    tri = lambda k: rs.triangular(0.9, 1.0, 1.1, k)  # noqa: E731  (Tri(lo, hi, mode=1))
    pop = {"Ua": tri(n), "Ca": hp.Ca * tri(n), "Cm": hp.Cm * tri(n), "Hm": hp.Hm * tri(n),
           "target": hp.target_temp + np.abs(rs.normal(0, 1, n)),
           "cap": rs.choice([12500.0, 15000.0, 17500.0], n)}
    ora = O.OracleEnv(props, random.Random(1), population=pop)
    acts = rs.randint(0, 2, (16, n)).astype(bool)
    t0 = time.perf_counter()
    ticks = 0
    while True:
        ora.step(acts[ticks % 16])
        ticks += 1
        el = time.perf_counter() - t0
        if el > budget_s:
            break
    return {"value": n * ticks / el, "unit": "house-steps/s", "cores": 1, "kind": "port",
            "sample": f"{n} houses x {ticks} ticks, random actions, oracle/env_np.py NumPy fp64 "
                      f"restatement (single thread) on the GPU box host, {el:.1f} s"}


def pmc_traffic(houses: int):
    """HBM bytes per k_step launch from the committed rocprofv3 PMC pass (profiles/), if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        rec = d.get(str(houses))
        return None if rec is None else float(rec["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = None
    kind = args.comm if args.comm != "default" else ("rccl" if world > 1 else "none")
    if world > 1 and kind == "none":
        raise SystemExit("--comm none needs WORLD_SIZE 1")
    if kind != "none":
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        from mdr_amd.distributed import make_comm

        comm = make_comm(kind)
    from mdr_amd.environment import Environment

    n_total = args.houses * world
    props = env_props(n_total)
    env = Environment(props, device=dev, rng=random.Random(4), population="synthetic", seed=1234,
                      rank=rank, world=world, comm=comm)
    n_loc = env.n_local
    chunk = min(args.chunk, args.steps)
    chunks = [chunk] * (args.steps // chunk) + ([args.steps % chunk] if args.steps % chunk else [])
    acts = None
    if args.mode == "buffer":
        acts = (torch.rand((chunk, n_loc), device=dev) < 0.5).to(torch.uint8)
    rew = torch.empty((chunk, n_loc), dtype=torch.float64, device=dev)
    dactor = None
    if args.workload == "actor":
        if world > 1:
            raise SystemExit("--workload actor runs on one GPU (sharded actor rollouts: see DESIGN.md)")
        from mdr_amd.actor import DeviceActor, make_actor

        dactor = DeviceActor(env, make_actor(env.obs_spec().n_feat, 2, [100, 100], seed=1),
                             precision=args.precision)

    def run(n):
        if dactor is not None:
            dactor.rollout(n, rewards=rew[:n])
        else:
            env.rollout(n, actions=None if acts is None else acts[:n], action_mode=args.mode,
                        rewards=rew[:n])

    # warmup: captures the graphs of every chunk size used below
    done = 0
    for c in sorted(set(chunks)):
        run(c)
        done += c
    while done < args.warmup:
        run(chunk)
        done += chunk
    torch.cuda.synchronize()

    def barrier():
        if comm is not None:
            import torch.distributed as dist

            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    # HIP events on the stream the k_step launches are issued on (the graph side stream)
    launch_stream = env.rollout_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(launch_stream)
    for c in chunks:
        run(c)
    ev1.record(launch_stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if comm is not None:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = n_total * args.steps / elapsed

    # dominant kernel k_step: one launch per tick (fused random controller + lookahead), so its
    # average launch duration over the timed region = launch-stream event time / steps (this
    # includes the ~1 us graph inter-kernel gap; rocprofv3's per-kernel average is in profiles/)
    per_tick_ms = gpu_ms / args.steps
    kern_ms, kern_launches = per_tick_ms, args.steps
    if comm is not None:
        # the sharded timed region also holds the per-tick RCCL allreduce: time k_step alone in
        # a local graph rollout of the same shard (after the timed region, rewards discarded)
        from mdr_amd._lib import ACT_RANDOM

        sh = env.shard
        ls = sh.launch_stream(True)
        kern_launches = min(args.steps, 500)
        ticks = env.driver_window(kern_launches)
        rbuf = rew[0]
        sh.rollout(ticks, None, 0, ACT_RANDOM, rbuf, 0, True)  # capture
        torch.cuda.synchronize()
        ev0.record(ls)
        sh.rollout(ticks, None, 0, ACT_RANDOM, rbuf, 0, True)
        ev1.record(ls)
        torch.cuda.synchronize()
        kern_ms = ev0.elapsed_time(ev1) / kern_launches
    if dactor is not None:
        # the rollout graph interleaves k_actor and k_step: time each kernel alone, back to back
        # on the current stream (HIP events on that stream), over the same state
        cur = torch.cuda.current_stream(dev)
        K = 50
        act_buf = torch.empty(n_loc, dtype=torch.uint8, device=dev)
        prob_buf = torch.empty(n_loc, dtype=torch.float32, device=dev)
        dactor.select_actions(action=act_buf, prob=prob_buf, count_next=False)
        torch.cuda.synchronize()
        ev0.record(cur)
        for _ in range(K):
            dactor.select_actions(action=act_buf, prob=prob_buf, count_next=False)
        ev1.record(cur)
        torch.cuda.synchronize()
        actor_ms = ev0.elapsed_time(ev1) / K
        kern_ms = max(per_tick_ms - actor_ms, 1e-6)  # the step kernel's share of a tick
    bytes_launch = BYTES_PER_HOUSE_STEP * n_loc
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic(n_loc)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "house-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device Philox population, reference noise model; fused Philox random actions)",
        "config": {"workload": "1M houses per GPU, random actions, fused FSM+thermal+reward step "
                               "(BASELINE metric at 1M houses; configs[1]'s controller)",
                   "houses_per_gpu": n_loc, "houses_total": n_total, "dt_s": props.time_step.seconds,
                   "signal": "sinusoidals", "penalty": "individual_L2", "action_mode": args.mode,
                   "chunk_ticks": chunk,
                   "sharded_pipeline": comm.pipeline(env.shard) if comm is not None else None,
                   "parallelism": f"house-sharded x{world} ({kind} allreduce of "
                                                        "per-tick power counts)" if comm is not None else "1 GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "kernel": step_kernel_name(n_loc, args.mode),
                     "kernel_avg_us": kern_ms * 1e3, "launches_timed": kern_launches,
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "bytes_per_house_step": BYTES_PER_HOUSE_STEP},
    }
    if dactor is not None:
        a = dactor.actor
        flops_house = 2 * sum(l.in_features * l.out_features for l in a.fc)  # 30,400 at F = 50
        flops_launch = flops_house * n_loc
        tfs = flops_launch / (actor_ms * 1e-3) / 1e12
        out["dtype"] = f"f64 env step + {args.precision} MFMA actor (fp32 accumulate)"
        out["data"] = ("synthetic (device Philox population, reference noise model); actor = the "
                       "reference MAPPO init (torch seed 1), actions sampled on device")
        out["config"]["workload"] = ("C5: 1M houses, MA-PPO actor select_actions fused with the obs "
                                     "(one launch) -> env.step (one launch) per tick, hipGraph chunks")
        out["config"]["action_mode"] = "mappo_actor"
        out["config"]["actor"] = {"layers": [a.fc[0].in_features, 100, 100, 2], "precision": args.precision}
        out["roofline"] = {"bound": "mfma", "achieved": tfs, "peak": BF16_PEAK_TFS, "unit": "TFLOP/s",
                           "frac": tfs / BF16_PEAK_TFS, "traffic": None, "kernel": "mdr::k_actor",
                           "kernel_avg_us": actor_ms * 1e3, "launches_timed": K,
                           "algorithmic_flops_per_launch": flops_launch, "flops_per_house": flops_house,
                           "mfma_products_per_mac": 3 if args.precision == "bf16x3" else 1,
                           "step_kernel": {"kernel": "mdr::k_step (BUFFER)", "avg_us": kern_ms * 1e3,
                                           "hbm_GBps": achieved, "frac": achieved / HBM_PEAK_GBS}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
