#!/usr/bin/env python
"""bench.py — vectorised env.step throughput (house-steps/s) on MI355X, with HBM roofline.

Workload (BASELINE.json metric "house-steps/s (env.step throughput) at 1M houses"): 1,048,576
houses — on one GPU configs[1]'s workload at the metric's size; under torchrun (WORLD_SIZE > 1)
config C4, the same 1,048,576-house cluster sharded over the GPUs (131,072 per GPU at 8: strong
scaling; --scaling weak keeps 1,048,576 per GPU) — with MARLconfig env_prop (dt = 4 s, L = 40 s,
individual_L2 rewards), sinusoidal regulation signal (perlin is parity-unpinned), synthetic
population drawn on device (Philox, the reference noise model), random actions from the fused
Philox controller (configs[1]'s controller).  A step = one env.step of every house: lockout FSM +
thermal update + cluster power + rewards (every tick's reward row is written), with the host
scalar drivers (outdoor temperature RNG, solar, signal) computed per tick inside the timed region.
Ticks are issued as rollout calls of up to --chunk ticks (mdr_rollout, direct launches), each
temporally blocked into windows of up to 32 ticks per launch (k_step_window; --window 0 = one
launch per tick); multi-GPU runs allreduce each window's cluster-power counts with RCCL inside the
loop (mdr_rollout_sharded, count-ahead pipeline).

Other workloads: --workload actor (config C5: MA-PPO actor fused with the obs, then env.step),
--workload greedy (config C3: device greedy-myopic controller, then env.step).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--houses H] [--chunk C] [--window W]
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
STATE_RW, PARAMS, REWARD, ACTION = 42, 48, 8, 1  # the §8(d) field sizes (bytes per house)
GREEDY_EXTRA = 26          # §8(d): + greedy key r/w 16, perm r/w 8, (P, lockout) gather 2
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s
BF16_PEAK_TFS = 2516.6     # dense bf16 MFMA: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (no sparsity)



def step_kernel_name(n_loc: int, mode: str, window: int, simple: bool = True, thermal: str = "affine") -> str:
    """The step kernel the library launches for this bench (mdr_capi.hip: window_launches /
    launch_step_on)."""
    if window > 0:  # the rocprofv3 spelling: k_step_window<ACT, HPT=2, SIMPLE, KA, FORM> (MDR_ACT_RANDOM = 1,
        # _BUFFER = 0; KA: the first window of a direct rollout call, drivers as kernel arguments — the
        # kernel-only timing below launches the KA = false instantiation, the same thermal loop; FORM:
        # MDR_THERMAL_AFFINE = 1, _EXACT = 0)
        return (f"void mdr::k_step_window<{1 if mode == 'random' else 0}, 2, {'true' if simple else 'false'}, "
                f"false, {1 if thermal == 'affine' else 0}>")
    tpw = 2 if n_loc <= 1572864 else 4  # mdr_capi.hip default_tpw
    act = "RANDOM,RANDOM" if mode == "random" else "BUFFER,0"
    return f"mdr::k_step_pipe<{tpw},{act}>"


def window_bytes(n: int, k: int, mode: str) -> int:
    """Algorithmic HBM bytes of one k_step_window launch of k ticks over n houses, in SURVEY
    §8(d)'s field sizes: state read+written once (42), parameters read once (48), one reward row
    per tick (8 k), plus the action rows for buffer mode (k)."""
    return n * (STATE_RW + PARAMS + REWARD * k + (ACTION * k if mode == "buffer" else 0))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--houses", type=int, default=1 << 20,
                    help="houses in the cluster (strong scaling, the default) or per GPU (--scaling weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="multi-GPU: strong = the --houses cluster sharded over the GPUs (config C4), weak = "
                         "--houses per GPU")
    ap.add_argument("--thermal", default="affine", choices=["affine", "exact"],
                    help="k_step_window's per-tick thermal update (mdr.h MDR_OPT_WINDOW_THERMAL)")
    ap.add_argument("--chunk", type=int, default=128, help="ticks per graph-captured rollout call")
    ap.add_argument("--window", type=int, default=32,
                    help="ticks per temporally blocked launch (k_step_window, <= 32); 0 = one launch per tick")
    ap.add_argument("--kernel-ticks", type=int, default=1024,
                    help="ticks per kernel-only timing call after the timed region (roofline.kernel_avg_us)")
    ap.add_argument("--kernel-reps", type=int, default=16,
                    help="kernel-only timing calls (16 x 1024 ticks = 512 timed launches of the 32-tick window kernel)")
    ap.add_argument("--kernel-warm-ticks", type=int, default=2048,
                    help="untimed kernel-only ticks before that timing (the GPU at its steady-state clock)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline time budget")
    ap.add_argument("--clock-warmup", type=float, default=0.0,
                    help="seconds of non-environment device work before the timed region (GPU clock ramp; "
                         "off by default: measured to slow the host side of a short timed region ~3x, "
                         "profiles/r02c_bench20_trace.log)")
    ap.add_argument("--host-spin-ms", type=float, default=0.0,
                    help="milliseconds of an idle host busy-loop right before the clock starts (diagnostics; measured "
                         "to slow a short timed call, so off by default)")
    ap.add_argument("--gc-off", action="store_true", help="diagnostics: disable Python's cyclic GC in the timed region")
    ap.add_argument("--min-warmup-calls", type=int, default=3,
                    help="warmup runs at least W steps AND at least this many rollout calls of the timed chunk "
                         "size (graph capture + 2 replays: the first replay of a graph and of the host path is "
                         "2-3x slower than the steady state, profiles/r02e_bench20_warmup.log)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gq-band", type=int, default=None, choices=[0, 1],
                    help="greedy: A/B of the predicted band (MDR_OPT_GQ_BAND; default on)")
    ap.add_argument("--step-tpw", type=int, default=None,
                    help="per-tick step kernel tiles per wave (MDR_OPT_STEP_TPW; default: the library's choice)")
    ap.add_argument("--above-mall-houses", type=int, default=16 << 20,
                    help="roofline.above_mall: the same step kernel timed alone at this many houses (working set "
                         "well above the 256 MB Infinity Cache, SURVEY 8(d) LLC caveat); 0 = skip")
    ap.add_argument("--trace", action="store_true",
                    help="print host phase timestamps of the timed region to stderr (diagnostics)")
    ap.add_argument("--graph", default="off", choices=["on", "off"],
                    help="rollout launch policy: off = Environment.rollout's default (direct launches, the first "
                         "window's drivers as kernel arguments), on = staged drivers + hipGraph replay")
    ap.add_argument("--mode", default="random", choices=["random", "buffer"])
    ap.add_argument("--workload", default="step", choices=["step", "actor", "greedy"],
                    help="step: env.step with fused random actions (the BASELINE metric); actor: "
                         "config C5, MA-PPO actor select_actions fused with the obs, then env.step; "
                         "greedy: config C3, device greedy-myopic controller then env.step")
    ap.add_argument("--precision", default="fp32", choices=["bf16x3", "fp32", "bf16"],
                    help="actor MFMA precision (--workload actor; fp32 = the reference Actor's)")
    ap.add_argument("--fp32-form", default="f16_split", choices=["f16_split", "bf16_split3"],
                    help="the fp32 precision's arithmetic (MDR_OPT_ACTOR_FP32_FORM)")
    ap.add_argument("--comm", default="default", choices=["default", "none", "rccl", "torch", "host"],
                    help="exchange for the sharded path (default: rccl when WORLD_SIZE > 1); "
                         "'rccl' at world 1 exercises the sharded C loop on one GPU; 'host' = the same C loops "
                         "with gloo collectives (ranks may share one GPU: a rehearsal of the multi-GPU line)")
    return ap.parse_args()


def env_props(n_total: int):
    from mdr_amd.config import EnvironmentProperties

    p = EnvironmentProperties.from_json(os.path.join(ROOT, "tests", "golden", "marl_env_prop.json"))
    p.cluster_prop.nb_agents = n_total
    p.power_grid_prop.signal_properties.mode = "sinusoidals"
    return p


def _synthetic_pop(props, n, seed):
    import numpy as np

    rs = np.random.RandomState(seed)
    hp = props.cluster_prop.house_prop
    tri = lambda k: rs.triangular(0.9, 1.0, 1.1, k)  # noqa: E731  (Tri(lo, hi, mode=1))
    return {"Ua": tri(n), "Ca": hp.Ca * tri(n), "Cm": hp.Cm * tri(n), "Hm": hp.Hm * tri(n),
            "target": hp.target_temp + np.abs(rs.normal(0, 1, n)),
            "cap": rs.choice([12500.0, 15000.0, 17500.0], n)}


def _cpu_run(job):
    """One CPU-baseline measurement in this process: (config, houses, seconds) ->
    (house-steps, elapsed s).  oracle/env_np.py (NumPy fp64, one thread)."""
    import numpy as np

    from oracle import env_np as O

    cfg, n, seconds = job
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    if cfg == "C5":  # MA-PPO: the oracle's norm_state_dict rows -> torch fp32 actor (batched) -> Categorical
        import torch

        from mdr_amd.actor import make_actor

        torch.set_num_threads(1)
        props = env_props(n)
        ora = O.OracleEnv(props, random.Random(1), population=_synthetic_pop(props, n, 0))
        actor = make_actor(ora.norm_vector().shape[1], 2, [100, 100], seed=1)
        gen = torch.Generator().manual_seed(3)

        def act():
            with torch.no_grad():
                p = actor(torch.from_numpy(ora.norm_vector()).float())
            return torch.multinomial(p, 1, generator=gen).squeeze(1).numpy().astype(bool)
    elif cfg == "C1":  # 50 houses, deadband bang-bang, reference population + RNG stream
        props = env_props(n)
        ora = O.OracleEnv(props, random.Random(4))
        hp = props.cluster_prop.house_prop
        act = lambda: O.deadband_bangbang(ora.T, ora.pop["target"], hp.deadband, ora.on)  # noqa: E731
    else:
        props = env_props(n)
        ora = O.OracleEnv(props, random.Random(1), population=_synthetic_pop(props, n, 0))
        if cfg == "C2":  # random actions
            rs = np.random.RandomState(1)
            acts = rs.randint(0, 2, (16, n)).astype(bool)
            act = lambda: acts[ticks % 16]  # noqa: E731
        else:  # C3: greedy-myopic on the post-step state, budget = the current signal
            cap = ora.pop["cap"]
            cop = props.cluster_prop.house_prop.hvac_prop.cop
            act = lambda: O.greedy(ora.T, ora.pop["target"], cap, cop, ora.lock, float(ora.S))  # noqa: E731
    ticks = 0
    t0 = time.perf_counter()
    while True:
        ora.step(act())
        ticks += 1
        el = time.perf_counter() - t0
        if el > seconds:
            return n * ticks, el


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(budget_s: float):
    """The oracle (oracle/env_np.py: NumPy fp64 restatement of the reference env step) timed on
    this host on bounded samples of BASELINE's configs: C1 (50 houses, deadband bang-bang), C2
    (65,536 houses, random actions: the bench workload's per-house work) and C3 (1,048,576 houses,
    greedy-myopic, one core: the algorithm is sequential), 1 core and all cores (independent
    processes, one per core, each stepping its own C2 sample).  The headline entry is C2 on all
    cores."""
    import multiprocessing as mp

    ncpu = os.cpu_count() or 1
    procs = max(1, min(ncpu, 16))  # the GPU box grants 16 cores to a job
    b = budget_s
    out = {"cpu_model": _cpu_model(), "os_cpu_count": ncpu, "configs": {}}
    hs, el = _cpu_run(("C1", 50, 0.15 * b))
    out["configs"]["C1_50_deadband_bbc_1core"] = {"value": hs / el, "ticks": hs // 50}
    hs, el = _cpu_run(("C2", 65536, 0.3 * b))
    c2_1 = hs / el
    out["configs"]["C2_65536_random_1core"] = {"value": c2_1, "ticks": hs // 65536}
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this process's GPU state
    pool = ctx.Pool(procs)
    try:
        res = pool.map(_cpu_run, [("C2", 65536, 0.3 * b)] * procs)
    finally:  # the workers exit on their own (no terminate(): no SIGTERM'd interpreters)
        pool.close()
        pool.join()
    c2_all = sum(h for h, _ in res) / max(e for _, e in res)
    out["configs"][f"C2_65536_random_{procs}cores"] = {"value": c2_all, "procs": procs}
    hs, el = _cpu_run(("C3", 1 << 20, 0.2 * b))
    out["configs"]["C3_1048576_greedy_1core"] = {"value": hs / el, "ticks": hs // (1 << 20)}
    hs, el = _cpu_run(("C5", 65536, 0.15 * b))
    out["configs"]["C5_65536_mappo_actor_1core"] = {
        "value": hs / el, "ticks": hs // 65536,
        "what": "oracle norm_vector rows -> torch fp32 Actor (batched forward, 1 thread) -> Categorical sample -> "
                "oracle step; the reference does N batch-1 forwards per tick (mappo.py:83-97), so this port is "
                "faster than the reference's own loop"}
    out["reference_itself"] = {"C1_50_deadband_bbc_1core": 31752, "unit": "house-steps/s",
                               "where": "the reference env (single-thread Python) in the survey container, "
                                        "Xeon 1 core (BASELINE.md:30, SURVEY.md section 6); it cannot run on the "
                                        "GPU box (the reference does not travel)"}
    out.update({"value": c2_all, "unit": "house-steps/s", "cores": procs, "kind": "port",
                "sample": f"oracle/env_np.py (NumPy fp64 restatement, 1 thread per process) on {procs} "
                          f"processes x 65,536 houses, random actions, {0.3 * b:.1f} s each "
                          f"(1 core: {c2_1:.3e}); host {out['cpu_model']}, os.cpu_count() = {ncpu}"})
    return out


def pmc_record(kernel: str, houses: int):
    """The committed rocprofv3 PMC record of `kernel` at `houses` (profiles/pmc_traffic.json,
    written by tools/collect_profiles.py: per-launch counter sums), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        rec = d.get(kernel, {}).get(str(houses))
        return rec if isinstance(rec, dict) else None
    except (OSError, ValueError, AttributeError):
        return None


def pmc_traffic(kernel: str, houses: int):
    """HBM bytes per launch of `kernel` at `houses` from the committed PMC passes, if collected."""
    rec = pmc_record(kernel, houses)
    try:
        return None if rec is None else float(rec["hbm_bytes_per_launch"])
    except (KeyError, TypeError, ValueError):
        return None


# wave64 VALU issue peak of MI355X: 256 CUs x 4 SIMDs, one wave64 instruction per 4 cycles per SIMD
# (16 lanes; fp64 FMA at full rate), 2.4 GHz peak engine clock (MI355X_MICROARCH.md)
VALU_PEAK_GINST = 1024 * 2.4 / 4.0  # G wave-instructions / s


def valu_roofline(kernel: str, houses: int, kern_ms: float):
    """The issue-rate roofline that actually bounds the temporally blocked step kernel (fp64 VALU):
    SQ_INSTS_VALU per launch from the committed PMC record over the live per-launch time."""
    rec = pmc_record(kernel, houses)
    if rec is None or "SQ_INSTS_VALU" not in rec or kern_ms <= 0:
        return None
    inst = float(rec["SQ_INSTS_VALU"])
    ach = inst / (kern_ms * 1e-3) / 1e9
    return {"achieved": ach, "peak": VALU_PEAK_GINST, "unit": "G wave64 VALU instr/s", "frac": ach / VALU_PEAK_GINST,
            "valu_instr_per_launch": inst,
            "source": "SQ_INSTS_VALU per launch (profiles/pmc_traffic.json) / kernel_avg_us; peak = 1024 SIMDs x "
                      "2.4 GHz / 4 cycles (the clock under this fp64 load is ~1.75 GHz, GRBM_GUI_ACTIVE)"}


def above_mall(houses: int, args, kern_1m: str) -> dict:
    """The dominant kernel timed ALONE at `houses` (16M by default: ~1.6 GB of state + parameters,
    ~6x the 256 MB Infinity Cache, so the fraction is HBM-honest), as for the 1M line: untimed
    warm ticks, then hipExtLaunchKernel events around every 32-tick k_step_window launch
    (mdr_time_step_kernels); traffic = the committed PMC record at that size."""
    import torch

    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    env = Environment(env_props(houses), device="cuda:0", rng=random.Random(4), population="synthetic", seed=1234)
    sh = env.shard
    kt = 32
    kern = step_kernel_name(houses, "random", 32, True, args.thermal)
    buf = torch.empty((kt, houses), dtype=torch.float64, device="cuda:0")
    for _ in range(4):  # warm: clock and caches in the state the timed launches see
        sh.rollout(env.driver_window(kt), None, 0, L.ACT_RANDOM, buf, houses, True)
    ms, launches = 0.0, 0
    for _ in range(8):
        m, l = sh.time_step_kernels(env.driver_window(kt), None, 0, L.ACT_RANDOM, buf, houses)
        ms += m
        launches += l
    kern_ms = ms / launches
    b = window_bytes(houses, kt, "random")
    achieved = b / (kern_ms * 1e-3) / 1e9
    del buf, env
    torch.cuda.empty_cache()
    return {"houses": houses, "kernel": kern, "same_kernel_as_1m": kern == kern_1m, "kernel_avg_us": kern_ms * 1e3,
            "launches_timed": launches, "algorithmic_bytes_per_launch": b, "achieved": achieved,
            "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(kern, houses),
            "timing": "hipExtLaunchKernel events around each 32-tick launch, 8 calls after 4 untimed ones"}


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)  # before this process touches the GPU
    if args.comm == "host":  # (rehearsal: the ranks may share the visible GPUs)
        local = local % max(1, torch.cuda.device_count())
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
        if kind == "host":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        from mdr_amd.distributed import make_comm

        comm = make_comm(kind)
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    n_total = args.houses * world if args.scaling == "weak" else args.houses
    props = env_props(n_total)
    env = Environment(props, device=dev, rng=random.Random(4), population="synthetic", seed=1234,
                      rank=rank, world=world, comm=comm)
    n_loc = env.n_local
    sh = env.shard
    window = min(max(args.window, 0), 32)
    sh.set_rollout_window(window)
    sh.set_option("window_thermal", L.THERMAL_AFFINE if args.thermal == "affine" else L.THERMAL_EXACT)
    chunk = min(args.chunk, args.steps)
    chunks = [chunk] * (args.steps // chunk) + ([args.steps % chunk] if args.steps % chunk else [])
    acts = None
    if args.mode == "buffer":
        acts = (torch.rand((chunk, n_loc), device=dev) < 0.5).to(torch.uint8)
    rew = torch.empty((chunk, n_loc), dtype=torch.float64, device=dev)
    dactor = None
    if args.workload == "actor":  # (sharded: the RCCL C loop with the ring-halo exchange per tick)
        from mdr_amd.actor import DeviceActor, make_actor

        dactor = DeviceActor(env, make_actor(env.obs_spec().n_feat, 2, [100, 100], seed=1),
                             precision=args.precision, fp32_form=args.fp32_form)
    g_act = None
    if args.workload == "greedy":
        if world > 1:
            raise SystemExit("--workload greedy runs on one GPU (config C3)")
        g_act = torch.empty(n_loc, dtype=torch.uint8, device=dev)
    if args.gq_band is not None:
        env.shard.set_option("gq_band", args.gq_band)
    if args.step_tpw is not None:  # (A/B of the per-tick step kernel's tiles per wave, MDR_OPT_STEP_TPW)
        env.shard.set_option("step_tpw", args.step_tpw)

    use_graph = args.graph == "on"

    def run(n):
        if dactor is not None:
            dactor.rollout(n, rewards=rew[:n])
        elif g_act is not None:  # C3: controller on the post-step state -> step, every tick, one C
            env.greedy_rollout(n, actions=g_act, rewards=rew[:n])  # call (the step writes the next keys)
        else:  # (whole buffers when the chunk fills them: no tensor views built per call)
            env.rollout(n, actions=None if acts is None else (acts if n == chunk else acts[:n]),
                        action_mode=args.mode, rewards=rew if n == chunk else rew[:n], use_graph=use_graph)

    # warmup: captures the graphs of every chunk size used below
    done = 0
    for c in sorted(set(chunks)):
        run(c)
        done += c
    calls = len(set(chunks))
    while done < args.warmup or calls < args.min_warmup_calls:
        run(chunk)
        done += chunk
        calls += 1
    warm_steps = done
    torch.cuda.synchronize()

    def barrier():
        if comm is not None:
            import torch.distributed as dist

            dist.barrier()

    if args.clock_warmup > 0:  # optional: unrelated device work (a buffer increment) before timing
        spin = torch.zeros(1 << 26, dtype=torch.float32, device=dev)
        t_spin = time.perf_counter()
        while time.perf_counter() - t_spin < args.clock_warmup:
            for _ in range(8):
                spin.add_(1.0)
            torch.cuda.synchronize()
        del spin
    barrier()
    torch.cuda.synchronize()
    # HIP events on the stream the step launches are issued on
    launch_stream = env.rollout_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for ev in (ev0, ev1):  # torch creates the HIP event on its first record(): not inside the timed region
        ev.record(launch_stream)
    torch.cuda.synchronize()
    trace = []
    if args.trace:  # wrap the two host phases of a rollout call with timestamps
        dw, ro = env.driver_window, sh.rollout

        def _dw(*a, **k):
            trace.append(("drivers>", time.perf_counter()))
            r = dw(*a, **k)
            trace.append(("drivers<", time.perf_counter()))
            return r

        def _ro(*a, **k):
            trace.append(("C call>", time.perf_counter()))
            r = ro(*a, **k)
            trace.append(("C call<", time.perf_counter()))
            return r

        env.driver_window, sh.rollout = _dw, _ro
    ev0.record(launch_stream)  # on the idle stream, before the clock starts (not part of a step)
    t_spin = time.perf_counter()
    while time.perf_counter() - t_spin < args.host_spin_ms * 1e-3:
        pass
    if args.gc_off:
        import gc

        gc.disable()
    t0 = time.perf_counter()
    for c in chunks:
        run(c)
    ev1.record(launch_stream)
    t_sub = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if args.gc_off:
        gc.enable()
    if args.trace:
        env.driver_window, sh.rollout = dw, ro
        print("trace (us from t0): " + ", ".join(f"{k} {1e6 * (t - t0):.1f}" for k, t in trace) +
              f", submitted {1e6 * (t_sub - t0):.1f}, synchronized {1e6 * (t1 - t0):.1f}", file=sys.stderr)
    barrier()
    elapsed = t1 - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if comm is not None:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if kind == "host" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = n_total * args.steps / elapsed

    # ---- roofline of the dominant kernel: timed ALONE after the timed region, >= 500 ticks in one
    # graph-captured local rollout (rewards kept: [ticks, n] rows), HIP events on its launch stream
    cur = torch.cuda.current_stream(dev)
    kt = max(args.kernel_ticks, 1)
    mode_id = L.ACT_RANDOM if args.mode == "random" else L.ACT_BUFFER
    simple = env.init_props.cluster_prop.house_prop.deadband == 0.0 and env._norm_temp == 1.0
    kern = step_kernel_name(n_loc, args.mode, window, simple, args.thermal)
    actor_ms = graph_ms = None
    if dactor is None and g_act is None:
        kbuf = torch.empty((kt, n_loc), dtype=torch.float64, device=dev)
        kacts = None if acts is None else (torch.rand((kt, n_loc), device=dev) < 0.5).to(torch.uint8)
        kticks = env.driver_window(kt)
        ls = sh.launch_stream()
        for rep in range(2):  # the whole graph (count, reduce and step kernels): capture, then a timed replay
            if rep:
                torch.cuda.synchronize()
                ev0.record(ls)
            sh.rollout(kticks, kacts, n_loc if kacts is not None else 0, mode_id, kbuf, n_loc, True)
        ev1.record(ls)
        torch.cuda.synchronize()
        graph_ms = ev0.elapsed_time(ev1)
        # the step kernel ALONE, in steady state: --kernel-warm-ticks untimed, then the same rollout
        # issued directly with hipExtLaunchKernel start/stop events around every step-kernel launch
        # (mdr_time_step_kernels), averaged over its launches
        for _ in range(max(args.kernel_warm_ticks, 0) // kt):
            sh.rollout(env.driver_window(kt), kacts, n_loc if kacts is not None else 0, mode_id, kbuf, n_loc, True)
        step_ms, launches = 0.0, 0
        for _ in range(max(args.kernel_reps, 1)):
            ms_r, l_r = sh.time_step_kernels(env.driver_window(kt), kacts, n_loc if kacts is not None else 0,
                                             mode_id, kbuf, n_loc)
            step_ms += ms_r
            launches += l_r
        del kbuf
        kern_ms = step_ms / launches
        k_win = kt * max(args.kernel_reps, 1) // launches if window > 0 else 1
        bytes_launch = window_bytes(n_loc, k_win, args.mode) if window > 0 else BYTES_PER_HOUSE_STEP * n_loc
        steps_launch = k_win
    elif g_act is not None:
        K = min(20, rew.shape[0])
        gt = env.driver_window(K)  # (the drivers first: the events bracket the device work)
        torch.cuda.synchronize()
        ev0.record(cur)
        sh.greedy_rollout(gt, g_act, 0, rew[:K], n_loc)
        ev1.record(cur)
        torch.cuda.synchronize()
        launches, kern_ms = K, ev0.elapsed_time(ev1) / K
        bytes_launch = (BYTES_PER_HOUSE_STEP + GREEDY_EXTRA) * n_loc
        steps_launch = 1
        kern = ("greedy tick: histogram select (k_gq_binsc, k_gq_finish; codes, superbin and predicted-band "
                "bin counts from the previous k_step_pipe's epilogue) + k_step_pipe")
    else:
        # the actor rollout graph interleaves k_actor and k_step: time the actor alone
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
        actor_status = dactor.status()  # (the headline launches: tiles left to the fp32 fallback, faults)
        # the other precisions / forms, timed the same way beside the headline one
        from mdr_amd.actor import DeviceActor

        beside = {}
        for name, kw in (("fp32_f16_split", {"precision": "fp32", "fp32_form": "f16_split"}),
                         ("fp32_bf16_split3", {"precision": "fp32", "fp32_form": "bf16_split3"}),
                         ("bf16x3", {"precision": "bf16x3"})):
            if kw["precision"] == args.precision and kw.get("fp32_form", args.fp32_form) == args.fp32_form:
                continue
            dx = DeviceActor(env, dactor.actor, **kw)
            dx.select_actions(action=act_buf, prob=prob_buf, count_next=False)
            torch.cuda.synchronize()
            ev0.record(cur)
            for _ in range(K):
                dx.select_actions(action=act_buf, prob=prob_buf, count_next=False)
            ev1.record(cur)
            torch.cuda.synchronize()
            beside[name] = ev0.elapsed_time(ev1) / K
        # (each DeviceActor loaded its weights into the shard: the headline actor again)
        env.shard.set_option("actor_fp32_form", L.FP32_F16_SPLIT if args.fp32_form == "f16_split" else L.FP32_BF16_SPLIT3)
        dactor.load_weights()
        launches = K
        kern_ms = max(gpu_ms / args.steps - actor_ms, 1e-6)  # the step kernel's share of a tick
        bytes_launch = BYTES_PER_HOUSE_STEP * n_loc
        steps_launch = 1
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic(kern, n_loc)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "house-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": warm_steps,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if world > 1 and args.scaling == "strong" else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device Philox population, reference noise model; fused Philox random actions)",
        "config": {"workload": (f"C4: {n_total:,} houses sharded over {world} GPUs ({n_loc:,} per GPU), random "
                                "actions, fused FSM+thermal+reward step, every tick's reward row written, one "
                                "allreduce of the window's power counts per window"
                                if world > 1 and args.scaling == "strong" else
                                f"{n_loc:,} houses per GPU, random actions, fused FSM+thermal+reward step, every "
                                "tick's reward row written (BASELINE metric at 1M houses; configs[1]'s controller)"),
                   "houses_per_gpu": n_loc, "houses_total": n_total, "dt_s": props.time_step.seconds,
                   "signal": "sinusoidals", "penalty": "individual_L2", "action_mode": args.mode,
                   "chunk_ticks": chunk, "window_ticks": window,
                   "sharded_pipeline": comm.pipeline(sh) if comm is not None else None,
                   "parallelism": f"house-sharded x{world} ({kind} allreduce of "
                                  "per-window power counts)" if comm is not None else "1 GPU"},
        "timed_region": {"wall_s": elapsed, "launch_stream_event_ms": gpu_ms,
                         "includes": "host drivers (OD-temperature RNG, solar, signal) + kernel launches ("
                                     + ("staged drivers, hipGraph replay" if args.graph == "on" else
                                        "direct: the first window's count, its drivers as step-kernel arguments, "
                                        "the later windows' drivers staged") + ") + device work",
                         "before": f"{warm_steps} warmup steps (>= the {args.warmup} requested and >= "
                                   f"{args.min_warmup_calls} rollout calls of the timed chunk size, until the "
                                   "host path is in steady state)" +
                                   (f" and {args.clock_warmup:.2f} s of non-environment device work"
                                    if args.clock_warmup > 0 else "") +
                                   (f"; a {args.host_spin_ms:g} ms idle host busy-loop" if args.host_spin_ms > 0 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kern,
                     "kernel_avg_us": kern_ms * 1e3, "launches_timed": launches,
                     "graph_us_per_launch": None if graph_ms is None else graph_ms * 1e3 / launches,
                     "house_steps_per_launch": steps_launch * n_loc,
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "bytes_per_house_step": bytes_launch / (steps_launch * n_loc),
                     "timing": f"hipExtLaunchKernel start/stop events around each step-kernel launch of {max(args.kernel_reps, 1)} "
                               f"{kt}-tick rollouts after the timed region and {args.kernel_warm_ticks} untimed kernel-only "
                               "ticks (steady-state clock)",
                     "valu": valu_roofline(kern, n_loc, kern_ms)},
    }
    if g_act is not None:
        out["data"] = "synthetic (device Philox population, reference noise model)"
        out["config"]["workload"] = ("C3: 1M houses, device GreedyMyopic (sort by -(T - target), budget = "
                                     "signal) on the post-step state, then env.step, every tick")
        out["config"]["action_mode"] = "greedy_myopic"
        out["roofline"]["timing"] = ("HIP events around one mdr_greedy_rollout call of 20 greedy+step ticks after "
                                     "the timed region (drivers computed before the first event)")
        gd = sh.greedy_diag()  # (after every timed call: it synchronises)
        out["greedy_select"] = {"calls": gd["calls"], "fallbacks": gd["fallbacks"],
                                "mean_window_houses": gd["window_sum"] / max(gd["calls"] - gd["fallbacks"], 1),
                                "last_window_houses": gd["window_last"]}
        bd = sh.greedy_band()  # the predicted band: calls whose bins pass k_gq_binsc skipped, and the misses
        out["greedy_select"]["band"] = {"skips": bd["skips"], "misses": bd["misses"], "band_base": bd["band_base"]}
        out["greedy_select"]["form"] = (
            "bins -> compact -> select every tick (--gq-band 0)" if args.gq_band == 0 else
            "adaptive band (the predicted band's two launches; budget jumps the host sees on bins -> compact -> "
            "select: MDR_OPT_GQ_ADAPTIVE); the fused one-launch tick MDR_OPT_GQ_FUSED is off (slower, DESIGN.md 3.3.1)")
    if dactor is not None:
        a = dactor.actor
        flops_house = 2 * sum(l.in_features * l.out_features for l in a.fc)  # 30,400 at F = 50
        flops_launch = flops_house * n_loc
        tfs = flops_launch / (actor_ms * 1e-3) / 1e12
        prec_name = ("fp32 (fp16 hi/lo split, 3 products on v_mfma_f32_16x16x32_f16)" if args.precision == "fp32"
                     and args.fp32_form == "f16_split" else "fp32 (three-way bf16 split, 6 products)"
                     if args.precision == "fp32" else args.precision)
        out["dtype"] = f"f64 env step + {prec_name} MFMA actor (fp32 accumulate)"
        out["data"] = ("synthetic (device Philox population, reference noise model); actor = the "
                       "reference MAPPO init (torch seed 1), actions sampled on device")
        out["config"]["workload"] = ("C5: 1M houses, MA-PPO actor select_actions fused with the obs "
                                     "(one launch) -> env.step (one launch) per tick, hipGraph chunks")
        out["config"]["action_mode"] = "mappo_actor"
        out["config"]["actor"] = {"layers": [a.fc[0].in_features, 100, 100, 2], "precision": args.precision,
                                  "fp32_form": args.fp32_form if args.precision == "fp32" else None,
                                  "status": actor_status}
        out["roofline"] = {"bound": "mfma", "achieved": tfs, "peak": BF16_PEAK_TFS, "unit": "TFLOP/s",
                           "frac": tfs / BF16_PEAK_TFS, "traffic": None, "kernel": "mdr::k_actor",
                           "kernel_avg_us": actor_ms * 1e3, "launches_timed": launches,
                           "algorithmic_flops_per_launch": flops_launch, "flops_per_house": flops_house,
                           "mfma_products_per_mac": {"bf16": 1, "bf16x3": 3,
                                                     "fp32": 3 if args.fp32_form == "f16_split" else 6}[args.precision],
                           "step_share": {"what": "launch-stream time per tick minus k_actor's time: the step "
                                                  "kernel's share of a tick (not a kernel duration)",
                                          "us_per_tick": kern_ms * 1e3}}
        out["roofline"]["beside"] = {
            name: {"kernel_avg_us": ms * 1e3, "achieved_tflops": flops_launch / (ms * 1e-3) / 1e12}
            for name, ms in beside.items()}
        out["roofline"]["beside"]["what"] = ("the same k_actor launches in the other arithmetic forms, timed the "
                                             "same way (fp32 = the reference Actor's precision)")
    if (dactor is None and g_act is None and rank == 0 and window > 0 and args.above_mall_houses > 0
            and args.mode == "random"):
        out["roofline"]["above_mall"] = above_mall(args.above_mall_houses, args, kern)
    out["build"] = {"lib": os.path.relpath(L.LIB_PATH, os.path.dirname(os.path.abspath(__file__))),
                    "src_hash": L.build_id(), "checked_against_tree": L.source_hash() == L.build_id()}
    if cpu is not None:
        # the headline CPU number of the line's own config: C2 (step), C3 (greedy), C5 (actor)
        key = {"greedy": "C3_1048576_greedy_1core", "actor": "C5_65536_mappo_actor_1core"}.get(args.workload)
        if key is not None:
            c = cpu["configs"][key]
            cpu = dict(cpu, value=c["value"], cores=1,
                       basis=("single core: the line's own config on 1 thread (the step line's value is C2 on 16 "
                              "processes; its 1-core C2 figure is configs.C2_65536_random_1core)"),
                       sample=(f"{key}: oracle/env_np.py (NumPy fp64, 1 thread)" +
                               (" + torch fp32 actor" if args.workload == "actor" else "") +
                               f", {c['ticks']} ticks; host {cpu['cpu_model']}"))
        else:
            cpu = dict(cpu, basis="16 processes x 1 thread of C2 (the 1-core figure: configs.C2_65536_random_1core)")
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        import torch.distributed as dist

        # deterministic teardown: every rank past its last collective, then the library's RCCL
        # communicator (mdr_destroy -> ncclCommDestroy) on every rank, then torch's process group
        torch.cuda.synchronize()
        dist.barrier()
        sh.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
