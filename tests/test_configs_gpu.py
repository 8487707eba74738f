"""BASELINE configs at their stated sizes, through the kernels the bench times.

* C2 workload at the benched size: ``rollout(64, 'random')`` at 1,048,576 houses (two launches of
  ``k_step_window``, the kernel in ``roofline.kernel``) == the one-launch-per-tick path bit for bit,
  and its first and last tick == the oracle (oracle/env_np.py) fed the exact Philox actions
  (tests/philox_np.py) on the device's input state;
* C4 per-rank size: the RCCL world-1 sharded rollout (``mdr_rollout_sharded``, count-ahead window
  pipeline: count + allreduce on the comm stream, reduce + step on the compute stream) at 131,072
  houses x 96 ticks (3 windows) == the oracle with replayed Philox actions, every tick;
* C5 at its size: ``DeviceActor.rollout`` at 1,048,576 houses == the select_actions / step_tensor
  loop; obs rows within 2 float32 ulps of the oracle's ``norm_vector`` on sampled houses;
  probabilities within the precision's tolerance of torch fp32 on the same rows.

Tolerances (BASELINE.json north_star: masks / counters bit-exact, T / P / reward within 1e-5):
on/lock/sso and P ``==``, temperatures rtol 1e-10, rewards rtol 1e-9 (fp64 in the reference's
operation order; only exp may differ by an ulp).
"""
import os
import random
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import golden_util as gu
import philox_np as PX
from oracle import env_np as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TEMP_RTOL = 1e-10
REW_RTOL = 1e-9
BENCH_SEED, BENCH_RNG = 1234, 4  # bench.py's population seed and driver RNG seed


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _props(n):
    return gu.props_from_overrides({"cluster_prop.nb_agents": n,
                                    "power_grid_prop.signal_properties.mode": "sinusoidals"})


def _pop(env):
    """The device population as the oracle's population dict (global order, this shard)."""
    prm = env.shard.host_params()
    caps = np.array(env._cap_values, np.float64)[prm["cap_idx"]]
    return {"Ua": prm["ua"], "Ca": prm["ca"], "Cm": prm["cm"], "Hm": prm["hm"], "target": prm["target"],
            "cap": caps}


def oracle_tick(props, pop, st, action, row):
    """One reference tick (environment.py:72-108 per-house part) from host state ``st`` with the
    tick drivers of a TickWindow row [t_od_prev, solar, s_prev, tick]: (new state, P, rewards)."""
    hp = props.cluster_prop.house_prop
    hv = hp.hvac_prop
    dt = props.time_step.seconds
    on, lock, sso = O.hvac_step(st["on"], st["lock"], st["sso"], action, hv.lockout_duration, dt)
    q = O.heat_transfer(on, pop["cap"], hv.latent_cooling_fraction)
    T, Tm = O.update_temperature(st["T"], st["Tm"], pop["Ua"], pop["Ca"], pop["Cm"], pop["Hm"], q,
                                 float(row[1]), float(row[0]), float(dt))
    P = float(np.sum(np.where(on, pop["cap"] / hv.cop, 0.0)))  # integers: exact in any order
    r = O.rewards(T, pop["target"], hp.deadband, P, float(row[2]), props.reward_prop, hp.target_temp)
    return {"on": on, "lock": lock, "sso": sso, "T": T, "Tm": Tm}, P, r


def _assert_state(got, ref, msg=""):
    for k in ("on", "lock", "sso"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} {msg}")
    np.testing.assert_allclose(got["T"], ref["T"], rtol=TEMP_RTOL, atol=0, err_msg=f"T {msg}")
    np.testing.assert_allclose(got["Tm"], ref["Tm"], rtol=TEMP_RTOL, atol=0, err_msg=f"Tm {msg}")


def _recording(env):
    """Wrap env._driver_window_vec (the vectorised drivers of driver_window and of rollout's one-C-call
    sequence) so every TickWindow a rollout computes is kept (its rows are the drivers the kernels
    consumed)."""
    rec = []
    orig = env._driver_window_vec

    def dwv(n, launch=None):
        out = orig(n) if launch is None else orig(n, launch)
        rec.append((out[0] if isinstance(out, tuple) else out).a.copy())
        return out

    env._driver_window_vec = dwv
    return rec


# ------------------------------------------------------------------------------------- C2 @ 1M
def test_benched_window_kernel_1m(torch_gpu):
    """The bench's workload and kernel at 1,048,576 houses: rollout(64) in ONE call (count,
    reduces, two k_step_window launches, the default affine thermal form) == the one-tick path
    (masks, counters, P ==; temperatures rtol 1e-10, rewards rtol 1e-9); its tick 0 and tick 63 ==
    the oracle on the device's input state with the replayed Philox actions."""
    torch = torch_gpu
    from mdr_amd.environment import Environment

    n, T = 1 << 20, 64
    props = _props(n)
    e1 = Environment(props, rng=random.Random(BENCH_RNG), population="synthetic", seed=BENCH_SEED)
    e2 = Environment(props, rng=random.Random(BENCH_RNG), population="synthetic", seed=BENCH_SEED)
    e2.shard.set_rollout_window(0)  # one launch per tick
    for e in (e1, e2):  # some history first: lockouts and a spread of temperatures
        e.rollout(37, action_mode="random", rewards=torch.empty(n, dtype=torch.float64, device="cuda"))
    pop = _pop(e1)
    st0 = e1.shard.host_state()
    rec = _recording(e1)
    tick0 = e1._tick
    R1 = e1.rollout(T, action_mode="random")  # the benched call shape
    assert len(rec) == 1 and rec[0].shape == (T, 4)
    R2a = e2.rollout(T - 1, action_mode="random")
    st62 = e2.shard.host_state()
    R2b = e2.rollout(1, action_mode="random")
    torch.cuda.synchronize()
    # the benched (affine) window form vs the one-tick kernels (the reference's expression): masks,
    # counters and P bit for bit, temperatures / rewards to the forms' rounding difference
    R2 = torch.cat([R2a, R2b]).cpu().numpy()
    np.testing.assert_allclose(R1.cpu().numpy(), R2, rtol=REW_RTOL, atol=1e-10)
    s1, s2 = e1.shard.host_state(), e2.shard.host_state()
    _assert_state(s1, s2, "window vs one-tick")
    assert e1._cluster_power() == e2._cluster_power()
    gids = np.arange(n, dtype=np.uint64)
    ticks = rec[0]
    # tick 0 from the state before the call
    _, P0, r0 = oracle_tick(props, pop, st0, PX.random_actions(BENCH_SEED, gids, tick0), ticks[0])
    np.testing.assert_allclose(R1[0].cpu().numpy(), r0, rtol=REW_RTOL, atol=1e-12, err_msg="reward tick 0")
    # tick 63 from the one-tick path's state after 63 ticks (== the window path's, above)
    assert int(ticks[T - 1:, 3].view(np.uint64)[0]) == tick0 + T - 1
    st63, P63, r63 = oracle_tick(props, pop, st62, PX.random_actions(BENCH_SEED, gids, tick0 + T - 1), ticks[T - 1])
    np.testing.assert_allclose(R1[T - 1].cpu().numpy(), r63, rtol=REW_RTOL, atol=1e-12, err_msg="reward tick 63")
    _assert_state(s1, st63, "after tick 63")
    assert e1._cluster_power() == P63
    assert P0 > 0 and np.all(np.isfinite(r63))


# -------------------------------------------------------------------------- C4 per-rank size
C4_N, C4_T = 131072, 96


def _c4_worker(rank, world, port, out_dir, pipeline):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "marl-demandresponse_amd"), os.path.dirname(HERE)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    import golden_util as g

    from mdr_amd.distributed import make_comm
    from mdr_amd.environment import Environment

    props = g.props_from_overrides({"cluster_prop.nb_agents": C4_N,
                                    "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, device=dev, rng=random.Random(BENCH_RNG), population="synthetic", seed=BENCH_SEED,
                      rank=rank, world=world, comm=make_comm("rccl"))
    env.shard.set_option("window_pipeline", 1 if pipeline else 0)
    prm = env.shard.host_params()
    st0 = env.shard.host_state()
    rec = _recording(env)
    tick0 = env._tick
    R = env.rollout(C4_T, action_mode="random")
    torch.cuda.synchronize()
    st = env.shard.host_state()
    np.savez(os.path.join(out_dir, "c4.npz"), R=R.cpu().numpy(), ticks=np.concatenate(rec), tick0=tick0,
             P=env._cluster_power(), cap_values=np.array(env._cap_values), **{"st0_" + k: v for k, v in st0.items()},
             **{"st_" + k: v for k, v in st.items()}, **{"prm_" + k: v for k, v in prm.items()})
    dist.destroy_process_group()


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("pipeline", [True, False])
def test_c4_rank_rccl_window_rollout_vs_oracle(tmp_path, pipeline):
    """C4's per-GPU shard (131,072 houses) through the RCCL sharded rollout at world 1: 96 ticks
    in one call = 3 windows of the count-ahead pipeline (or the one-stream order) == the oracle
    stepping the same Philox actions, every tick's rewards and the final state."""
    mp.start_processes(_c4_worker, args=(1, _free_port(), str(tmp_path), pipeline), nprocs=1, join=True,
                       start_method="spawn")
    d = np.load(tmp_path / "c4.npz")
    props = _props(C4_N)
    caps = d["cap_values"][d["prm_cap_idx"]]
    pop = {"Ua": d["prm_ua"], "Ca": d["prm_ca"], "Cm": d["prm_cm"], "Hm": d["prm_hm"], "target": d["prm_target"],
           "cap": caps}
    st = {k: d["st0_" + k] for k in ("T", "Tm", "on", "lock", "sso")}
    ticks = d["ticks"]
    assert ticks.shape == (C4_T, 4)
    gids = np.arange(C4_N, dtype=np.uint64)
    tick0 = int(d["tick0"])
    P = None
    for t in range(C4_T):
        st, P, r = oracle_tick(props, pop, st, PX.random_actions(BENCH_SEED, gids, tick0 + t), ticks[t])
        np.testing.assert_allclose(d["R"][t], r, rtol=REW_RTOL, atol=1e-12, err_msg=f"reward t={t}")
    _assert_state({k: d["st_" + k] for k in ("T", "Tm", "on", "lock", "sso")}, st, "final")
    assert float(d["P"]) == P


# ------------------------------------------------------------------------------------- C5 @ 1M
@pytest.mark.parametrize("precision,atol", [("bf16x3", 1e-4), ("fp32", 4e-6), ("fp32_bf16", 4e-6)])
def test_c5_actor_rollout_1m(torch_gpu, precision, atol):
    """C5's actor path at 1,048,576 houses: DeviceActor.rollout (actor -> step per tick, one graph)
    == the select_actions / step_tensor loop over 4 ticks (actions, probabilities, rewards, state);
    at every tick the loop's obs rows are within 2 float32 ulps of the oracle's norm_vector on
    8,192 sampled houses (incl. both ring ends) and its probabilities within ``atol`` of torch fp32
    (bf16x3 1e-4, fp32 4e-6 in both its forms: the fp16 split, default, and the three-way bf16
    split, 'fp32_bf16').  The actor is the seed-1 reference actor with the obs normalisation
    folded into layer 1 (golden_util.calibrated_actor): at 1M houses the raw seed-1 policy
    saturates (the cluster-power feature is ~0.4 N, norm.py:145), and a probability check would
    compare 1.0 with 1.0; here most probabilities lie in (0.05, 0.95) and both actions occur."""
    torch = torch_gpu
    from mdr_amd.actor import DeviceActor
    from mdr_amd.environment import Environment

    n, T = 1 << 20, 4
    props = _props(n)
    ea = Environment(props, rng=random.Random(BENCH_RNG), population="synthetic", seed=BENCH_SEED)
    eb = Environment(props, rng=random.Random(BENCH_RNG), population="synthetic", seed=BENCH_SEED)
    F = ea.obs_spec().n_feat
    actor = gu.calibrated_actor(F, ea.obs_tensor().abs().amax(0).double().cpu().numpy(), seed=1).to("cuda")
    kw = {"precision": "fp32", "fp32_form": "bf16_split3"} if precision == "fp32_bf16" else {"precision": precision}
    da, db = DeviceActor(ea, actor, **kw), DeviceActor(eb, actor, **kw)
    rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
    acts = torch.empty((T, n), dtype=torch.uint8, device="cuda")
    probs = torch.empty((T, n), dtype=torch.float32, device="cuda")
    da.rollout(T, rewards=rew, actions=acts, probs=probs)
    pop = _pop(eb)
    k = ea.obs_spec().n_comm
    lo, hi = k // 2, (k + 1) // 2
    rs = np.random.RandomState(5)
    sample = np.unique(np.concatenate([np.arange(8), np.arange(n - 8, n), rs.randint(0, n, 8176)]))
    offs = np.array([j - lo for j in range(lo)] + [1 + j for j in range(hi)], np.int64)
    links = (sample[:, None] + offs[None, :]) % n  # the 'neighbours' ring rows of the sampled houses
    obs = torch.empty((n, F), dtype=torch.float32, device="cuda")
    pr = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    for t in range(T):
        a, p = db.select_actions(probs=pr, obs_out=obs, count_next=True)
        # the obs rows this tick's actions were drawn from, against the oracle on the same state
        st = eb.shard.host_state()
        o = {"T": st["T"], "Tm": st["Tm"], "on": st["on"], "lock": st["lock"], "sso": st["sso"],
             "P": eb._cluster_power(), "S": float(eb.power_grid.current_signal), "Tod": float(eb.current_od_temp),
             "G": float(eb._solar)}
        ref = O.norm_vector_rows(props, pop, o, sample, links)
        got = obs.cpu().numpy()[sample]
        np.testing.assert_array_max_ulp(got, ref.astype(np.float32), maxulp=2)
        with torch.no_grad():
            tp = actor(obs[torch.from_numpy(sample).to("cuda")]).cpu().numpy()
        got_p = pr.cpu().numpy()[sample]
        assert float(np.abs(got_p - tp).max()) < atol, (t, float(np.abs(got_p - tp).max()))
        gu.assert_not_saturated(got_p[:, 1])
        r = eb.step_tensor(a)
        assert torch.equal(a, acts[t]), t
        assert torch.equal(p, probs[t]), t
        assert torch.equal(r, rew[t]), t
    for key in ("t_air", "t_mass", "hvac"):
        assert torch.equal(getattr(ea.shard, key), getattr(eb.shard, key)), key
    assert ea._cluster_power() == eb._cluster_power()
    gu.assert_not_saturated(probs.cpu().numpy(), acts.cpu().numpy())
    assert da.status()["range_faults"] == 0 and db.status()["range_faults"] == 0
