"""Greedy histogram-select state per call: the single-shard form and the sharded form (RCCL world 1,
the stages run with collectives to self) on the tick script of tests/test_distributed_gpu.py.

    python tools/gq_probe.py [--houses 3001]
"""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd"), os.path.join(ROOT, "tests")]


def script(env, n_total, torch, dev, sharded):
    import numpy as np

    lo, nl = env._offset, env.n_local
    for _ in range(5):
        env.step_tensor(None, action_mode="random", lookahead="random")
    for t in range(3):
        a = np.random.RandomState(100 + t).randint(0, 2, n_total).astype(np.uint8)[lo:lo + nl]
        env.step_tensor(torch.from_numpy(a).to(dev))
    out = []
    for t in range(2):
        sh = env.shard
        S = float(env.power_grid.current_signal)
        if sharded:
            act = torch.empty(nl, dtype=torch.uint8, device=dev)
            v = sh.gq_shard_begin()
            print("  begin", sh.greedy_state(), "range", v["range"].cpu().tolist())
            env._comm.allreduce_count32(sh, v["super"])
            env._comm.allreduce_min(sh, v["range"])
            sh.gq_shard_bins(S)
            print("  bins ", sh.greedy_state())
            env._comm.allreduce_count32(sh, v["bins"])
            sh.gq_shard_compact(S, act)
            print("  compact", sh.greedy_state(), "header", v["window"][:16].view(torch.int32).cpu().tolist())
            g = env._comm.allgather_bytes(sh, v["window"])
            sh.gq_shard_select(S, g, env.world, act)
            print("  select", sh.greedy_state(), "fallback", sh.gq_shard_fallback())
        else:
            act = env.greedy_actions()
            print("  single", sh.greedy_state())
        print(f" tick {t}: S={S} taken={int(act.sum())}")
        out.append(act.cpu().numpy().copy())
        env.step_tensor(act)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=3001)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    import numpy as np
    import torch
    import torch.distributed as dist

    import golden_util as gu
    from test_distributed_gpu import _overrides
    from mdr_amd.distributed import make_comm
    from mdr_amd.environment import Environment

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    props = gu.props_from_overrides(_overrides(a.houses, "individual_L2"))
    print("single shard")
    env = Environment(props, device=dev, rng=random.Random(4), population="synthetic", seed=77)
    r1 = script(env, a.houses, torch, dev, False)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    print("sharded, RCCL world 1")
    env2 = Environment(gu.props_from_overrides(_overrides(a.houses, "individual_L2")), device=dev,
                       rng=random.Random(4), population="synthetic", seed=77, rank=0, world=1,
                       comm=make_comm("rccl"))
    r2 = script(env2, a.houses, torch, dev, True)
    for t, (x, y) in enumerate(zip(r1, r2)):
        print(f"tick {t}: actions equal {bool(np.array_equal(x, y))}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
