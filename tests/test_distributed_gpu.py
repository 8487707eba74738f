"""Sharded device path on the GPU: the house-sharded Environment (one process per rank) must
reproduce the single-process run on the same seeds.

* world 1 over the library's own RCCL communicator (backend 'nccl'): exercises mdr_rccl_init,
  mdr_rccl_allreduce and the C rollout loop mdr_rollout_sharded on a real device: the count-ahead
  window pipeline (default) and its one-stream form, the per-tick loop serial and overlapped
  (reward written one launch later);
* world 2 over torch.distributed/gloo (TorchComm) with both ranks on cuda:0: exercises the
  sharding, the per-tick count / penalty allreduces and the ring-halo observation exchange with
  the HIP kernels (RCCL cannot put two ranks on one GPU; the 8-GPU RCCL run is the driver's).

Integers (on/lock/sso, counts, hence P) and everything derived per house in fp64 are bit-exact;
the common penalty modes reduce the cluster penalty in a different order per shard, so rewards
there are compared to 1e-12.
"""
import os
import random
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import golden_util as gu

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
T_STEP, T_BUF, T_GREEDY, T_ROLL = 5, 3, 2, 70  # 3 windows


INTERP = "interp"  # mode suffix: interpolation base power (row a10), re-estimated every 3 ticks


def _overrides(n, mode):
    pen, _, extra = mode.partition("+")
    o = {"cluster_prop.nb_agents": n, "power_grid_prop.signal_properties.mode": "sinusoidals",
         "reward_prop.penalty_props.mode": pen, "reward_prop.penalty_props.alpha_common_max": 0.5}
    if extra == INTERP:
        o.update({gu.BPP + "mode": "interpolation", gu.BPP + "interp_update_period": 12,
                  gu.BPP + "interp_nb_agents": 200})
    elif extra in ("closed_groups", "random_fixed"):  # table comm modes (sharded: all-gathered messages)
        o["cluster_prop.agents_comm_prop.mode"] = extra
    return o


def _run(env, n_total, torch, dev):
    """Fixed tick script: fused random steps, buffer steps, greedy steps, a rollout (individual_L2 only)."""
    lo, nl = env._offset, env.n_local
    rewards = []
    for _ in range(T_STEP):
        rewards.append(env.step_tensor(None, action_mode="random", lookahead="random").cpu().numpy().copy())
    for t in range(T_BUF):
        a = np.random.RandomState(100 + t).randint(0, 2, n_total).astype(np.uint8)[lo:lo + nl]
        rewards.append(env.step_tensor(torch.from_numpy(a).to(dev)).cpu().numpy().copy())
    for t in range(T_GREEDY):  # GreedyMyopic over the whole cluster (sharded: the histogram form)
        rewards.append(env.step_tensor(env.greedy_actions()).cpu().numpy().copy())
        if os.environ.get("MDR_TEST_GQ_DIAG"):
            print("greedy", env._offset, t, env.shard.greedy_state(), flush=True)
    if env.shard.penalty_mode == 0:
        r = env.rollout(T_ROLL, action_mode="random")
        rewards.extend(r.cpu().numpy().copy())
        for k in (20, 32):  # single windows: library RCCL -> begin (count + allreduce + P-only reduce) + KA step
            rewards.extend(env.rollout(k, action_mode="random").cpu().numpy().copy())
    st = env.shard.host_state()
    obs = env.obs_tensor().cpu().numpy().copy()
    return {"rewards": np.array(rewards), "T": st["T"], "Tm": st["Tm"], "on": st["on"], "lock": st["lock"],
            "sso": st["sso"], "P": env._cluster_power(), "obs": obs, "gq_fb": env._gq_shard_fallbacks}


def _variant(env, kind):
    """The launch form a test kind selects (mdr_set_option), on the sharded env and its reference:
    <comm>-winserial = windows without the count-ahead pipeline (one stream); <comm>-serial /
    <comm>-overlap = the per-tick C loop (window 0), serial or two-stream.  <comm> = rccl (the
    library's RCCL communicator) or host (the same C loops, collectives by torch.distributed
    callbacks: mdr_comm_host)."""
    form = kind.partition("-")[2]
    if kind == "torch":  # TorchComm steps every tick from Python (one-tick kernels): the exact form
        env.shard.set_option("window_thermal", 0)
    elif form == "winserial":
        env.shard.set_option("window_pipeline", 0)
    elif form in ("serial", "overlap"):
        env.shard.set_rollout_window(0)
        env.shard.set_option("sharded_overlap", form == "overlap")


def _comm_kind(kind):
    return kind.partition("-")[0]


def _worker(rank, world, port, backend, kind, n, mode, out_dir):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "marl-demandresponse_amd"), os.path.dirname(HERE)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    import golden_util as g

    from mdr_amd.distributed import make_comm
    from mdr_amd.environment import Environment

    env = Environment(g.props_from_overrides(_overrides(n, mode)), device=dev, rng=random.Random(4),
                      population="synthetic", seed=77, rank=rank, world=world,
                      comm=make_comm(_comm_kind(kind)))
    _variant(env, kind)
    if kind.startswith("rccl"):  # world 1: the sharded greedy stages with RCCL collectives to self
        env._gq_force_sharded = True
    res = _run(env, n, torch, dev)
    res["lo"] = env._offset
    if world > 1 and _comm_kind(kind) == "host":
        #  config C3's one-call loop refuses a sharded context: a shard-local decision
        # and step would use shard-local counts (Environment.greedy_rollout takes the per-tick loop)
        from mdr_amd._lib import MdrError

        a = torch.empty(env.n_local, dtype=torch.uint8, device=dev)
        r = torch.empty(env.n_local, dtype=torch.float64, device=dev)
        try:
            env.shard.greedy_rollout(env.driver_window(1), a, 0, r, 0)
            res["gr_guard"] = 0
        except MdrError as e:
            res["gr_guard"] = int("single-GPU only" in str(e))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    torch.cuda.synchronize()
    dist.destroy_process_group()


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("backend,kind,world,n,mode", [
    ("nccl", "rccl", 1, 3001, "individual_L2"),
    ("nccl", "rccl-winserial", 1, 3001, "individual_L2"),
    ("nccl", "rccl-serial", 1, 3001, "individual_L2"),
    ("nccl", "rccl-overlap", 1, 3001, "individual_L2"),
    ("gloo", "torch", 2, 3001, "individual_L2"),
    ("gloo", "torch", 2, 2048, "common_L2"),
    ("nccl", "rccl", 1, 3001, "individual_L2+interp"),
    ("gloo", "torch", 2, 3001, "individual_L2+interp"),
    ("gloo", "torch", 2, 2992, "individual_L2+closed_groups"),
    ("gloo", "torch", 2, 3001, "common_L2+random_fixed"),
    ("nccl", "rccl", 1, 131072, "individual_L2"),    # C4's per-GPU shard size
    ("gloo", "torch", 2, 262144, "individual_L2"),   # two C4-sized shards on cuda:0
    # distinct left / right peers (world >= 3): the point-to-point ring halo, uneven shards, the
    # greedy's window all-gather over 3..8 windows
    ("gloo", "torch", 3, 3001, "individual_L2"),
    ("gloo", "torch", 4, 2992, "individual_L2+closed_groups"),
    ("gloo", "torch", 4, 4096, "common_L2"),
    # the library's sharded C loops (count-ahead window pipeline, per-tick loops) at world 2..8,
    # collectives through torch.distributed callbacks (mdr_comm_host)
    ("gloo", "host", 2, 3001, "individual_L2"),
    ("gloo", "host", 3, 3001, "individual_L2"),
    ("gloo", "host-winserial", 3, 3001, "individual_L2"),
    ("gloo", "host-serial", 3, 3001, "individual_L2"),
    ("gloo", "host-overlap", 3, 3001, "individual_L2"),
    ("gloo", "host", 4, 4 * 131072, "individual_L2"),  # half the C4 cluster, C4-sized shards
    ("gloo", "host", 8, 8 * 131072, "individual_L2"),  # C4: the 1,048,576-house cluster on 8 ranks
])
def test_sharded_equals_single(tmp_path, backend, kind, world, n, mode):
    import torch

    from mdr_amd.environment import Environment

    mp.start_processes(_worker, args=(world, _free_port(), backend, kind, n, mode, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    parts = sorted((np.load(tmp_path / f"rank{r}.npz") for r in range(world)), key=lambda p: int(p["lo"]))
    dev = torch.device("cuda", 0)
    env = Environment(gu.props_from_overrides(_overrides(n, mode)), device=dev, rng=random.Random(4),
                      population="synthetic", seed=77)
    _variant(env, kind)
    ref = _run(env, n, torch, dev)
    for key in ("on", "lock", "sso", "T", "Tm"):
        np.testing.assert_array_equal(np.concatenate([p[key] for p in parts]), ref[key], err_msg=key)
    got_r = np.concatenate([p["rewards"] for p in parts], axis=1)
    if mode.startswith("individual_L2"):
        np.testing.assert_array_equal(got_r, ref["rewards"])
    else:
        np.testing.assert_allclose(got_r, ref["rewards"], rtol=1e-12, atol=1e-15)
    for p in parts:
        assert float(p["P"]) == ref["P"]
        # the sharded histogram select decided every greedy tick (its results are checked above
        # either way); r03's occasional hand-off to the all-gather form was a race in
        # k_gq_compact (block 0 overwrote the crossing base the other blocks were still reading)
        assert int(p["gq_fb"]) == 0, int(p["gq_fb"])
        if world > 1 and _comm_kind(kind) == "host":
            assert int(p["gr_guard"]) == 1
    obs = np.concatenate([p["obs"] for p in parts])
    np.testing.assert_array_equal(obs, ref["obs"])


# ---------------------------------------------------------------- sharded MA-PPO rollout (C5)
T_ACT = 12


def _actor_run(env, torch, dist=None, layers=(100, 100)):
    from mdr_amd.actor import DeviceActor

    # the seed-1 reference actor with the obs normalisation folded into layer 1 (not saturated at
    # any cluster size); the scales are the cluster-wide feature maxima, identical on every rank
    m = env.obs_tensor().abs().amax(0).double().contiguous()
    if dist is not None:
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
    m = m.cpu().numpy()
    da = DeviceActor(env, gu.calibrated_actor(env.obs_spec().n_feat, m, seed=1, layers=layers).to(env.shard.device))
    nl = env.n_local
    A = torch.zeros((T_ACT, nl), dtype=torch.uint8, device=env.shard.device)
    Pr = torch.zeros((T_ACT, nl), dtype=torch.float32, device=env.shard.device)
    R = da.rollout(T_ACT, actions=A, probs=Pr)
    torch.cuda.synchronize()
    st = env.shard.host_state()
    return {"rewards": R.cpu().numpy(), "actions": A.cpu().numpy(), "probs": Pr.cpu().numpy(),
            "T": st["T"], "on": st["on"], "sso": st["sso"], "P": env._cluster_power()}


def _actor_worker(rank, world, port, backend, kind, n, out_dir, force_halo, layers):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "marl-demandresponse_amd"), os.path.dirname(HERE)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    import golden_util as g

    from mdr_amd.distributed import make_comm
    from mdr_amd.environment import Environment

    env = Environment(g.props_from_overrides(_overrides(n, "individual_L2")), device=dev, rng=random.Random(4),
                      population="synthetic", seed=77, rank=rank, world=world, comm=make_comm(_comm_kind(kind)))
    if force_halo:
        env.shard.set_option("force_halo", 1)
    if "-twocoll" in kind:  # MDR_OPT_HALO_IN_COUNTS off: a ring-halo send/recv + the count allreduce per tick
        env.shard.set_option("halo_in_counts", 0)
    if kind.endswith("-serialhalo"):  # (two collectives) MDR_OPT_HALO_OVERLAP off: halo, then one k_actor per tick
        env.shard.set_option("halo_overlap", 0)
    res = _actor_run(env, torch, dist, layers)
    res["lo"] = env._offset
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("backend,kind,world,force_halo,n,layers", [
    ("nccl", "rccl", 1, False, 3001, (100, 100)),   # C loop: actor -> RCCL count allreduce -> step
    # + the halo: the edge rows of the next tick summed into the count allreduce (to self), and the
    # two-collective form (ring-halo pack / ncclSend / ncclRecv to self, then the allreduce)
    ("nccl", "rccl", 1, True, 3001, (100, 100)),
    ("nccl", "rccl-twocoll", 1, True, 3001, (100, 100)),
    ("gloo", "torch", 2, False, 3001, (100, 100)),  # two shards on cuda:0, per-tick Python loop, P2P halo
    ("gloo", "torch", 3, False, 3001, (100, 100)),  # distinct left / right peers
    # the C loop, ONE collective per tick: actor -> edge rows of the post-step state (k_halo_step_pack)
    # -> allreduce of [count slab | every rank's rows] -> step
    ("gloo", "host", 3, False, 3001, (100, 100)),
    ("gloo", "host", 3, False, 3001, (64, 64, 64)),  # the layer chain (k_obs reads the halo) in the C loop
    # the two-collective C loop: halo on the side stream beside the interior tiles, or serial
    ("gloo", "host-twocoll", 3, False, 3001, (100, 100)),
    ("gloo", "host-twocoll-serialhalo", 3, False, 3001, (100, 100)),
    ("gloo", "host-twocoll", 3, False, 3001, (64, 64, 64)),
    # ragged shards around the interior / edge tile split: 994 = 32 * 31 + 2 houses per rank (the
    # second-to-last tile's ring reaches the next shard, so the halo overlap must stay off), 992
    # (whole tiles), 101 = 32 * 3 + 5 (four tiles, the last one holding hi houses)
    ("gloo", "host", 3, False, 3 * 994, (100, 100)),
    ("gloo", "host-twocoll", 3, False, 3 * 994, (100, 100)),
    ("gloo", "host-twocoll-serialhalo", 3, False, 3 * 994, (100, 100)),
    ("gloo", "host-twocoll", 3, False, 3 * 992, (100, 100)),
    ("gloo", "host-twocoll", 3, False, 3 * 101, (100, 100)),
    ("gloo", "host", 8, False, 8 * 131072, (100, 100)),  # C5: the 1,048,576-house cluster on 8 ranks
    ("gloo", "host-twocoll", 8, False, 8 * 131072, (100, 100)),
])
def test_sharded_actor_rollout_equals_single(tmp_path, backend, kind, world, force_halo, n, layers):
    """Sharded MA-PPO rollout (config C5) == the single-process graph rollout: actions, sampled
    probabilities, rewards, state and P bit for bit."""
    import torch

    from mdr_amd.environment import Environment

    mp.start_processes(_actor_worker, args=(world, _free_port(), backend, kind, n, str(tmp_path), force_halo, layers),
                       nprocs=world, join=True, start_method="spawn")
    parts = sorted((np.load(tmp_path / f"rank{r}.npz") for r in range(world)), key=lambda p: int(p["lo"]))
    env = Environment(gu.props_from_overrides(_overrides(n, "individual_L2")), device=torch.device("cuda", 0),
                      rng=random.Random(4), population="synthetic", seed=77)
    ref = _actor_run(env, torch, layers=layers)
    for key in ("actions", "probs", "rewards"):
        np.testing.assert_array_equal(np.concatenate([p[key] for p in parts], axis=1), ref[key], err_msg=key)
    for key in ("T", "on", "sso"):
        np.testing.assert_array_equal(np.concatenate([p[key] for p in parts]), ref[key], err_msg=key)
    for p in parts:
        assert float(p["P"]) == ref["P"]
    gu.assert_not_saturated(ref["probs"], ref["actions"])
