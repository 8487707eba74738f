"""A/B of the greedy tick's forms on config C3 (1M houses, bench.py's population) per power signal
(DESIGN §3.3's table): HIP events around mdr_greedy_rollout calls of K ticks, the forms alternating
on one context per signal (the drivers are computed before each call's first event):

  fused   MDR_OPT_GQ_FUSED 1 (producer epilogue -> k_gq_decide2 -> k_step_pipe GQ 2)
  band    MDR_OPT_GQ_FUSED 0, MDR_OPT_GQ_BAND 1, MDR_OPT_GQ_ADAPTIVE 0 (k_gq_binsc skips its bins pass on a hit)
  adaptive  the band form, ticks with a budget jump on the three-launch form (MDR_OPT_GQ_ADAPTIVE 1)
  noband  MDR_OPT_GQ_FUSED 0, MDR_OPT_GQ_BAND 0 (bins -> compact -> select every tick)

Prints per-tick medians, and the hit / miss counts of the band and of the fused decision.

    python tools/greedy_ab.py [reps] [ticks] [signals, comma-separated]
"""
import os
import random
import time
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "marl-demandresponse_amd"))

import torch  # noqa: E402

from bench import env_props  # noqa: E402
from mdr_amd.environment import Environment  # noqa: E402

FORMS = {"fused": {"gq_fused": 1}, "band": {"gq_fused": 0, "gq_band": 1, "gq_adaptive": 0},
         "adaptive": {"gq_fused": 0, "gq_band": 1, "gq_adaptive": 1}, "noband": {"gq_fused": 0, "gq_band": 0}}


def run_signal(signal, reps, K, n=1 << 20):
    props = env_props(n)
    props.power_grid_prop.signal_properties.mode = signal
    env = Environment(props, device="cuda:0", rng=random.Random(4), population="synthetic", seed=1234)
    sh = env.shard
    act = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rew = torch.empty(n, dtype=torch.float64, device="cuda:0")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {f: [] for f in FORMS}
    cnt = {f: [0, 0] for f in FORMS}  # hits, misses
    for form, opts in FORMS.items():  # warm every form: keys, maps, band in steady state
        for k, v in opts.items():
            sh.set_option(k, v)
        env.greedy_rollout(60, actions=act, rewards=rew)
    for r in range(reps):
        for form, opts in FORMS.items():
            for k, v in opts.items():
                sh.set_option(k, v)
            # a form switch restarts the form's key map from its last call's (stale: the state moved
            # on under the other forms; the first call may fall back to gq_exact): re-warm untimed
            env.greedy_rollout(8, actions=act, rewards=rew)
            ticks = env.driver_window(K)
            b0, f0, g0 = sh.greedy_band(), sh.greedy_fused_diag(), sh.greedy_diag()
            torch.cuda.synchronize()
            ev0.record()
            h0 = time.perf_counter()
            sh.greedy_rollout(ticks, act, 0, rew, 0)
            host_us = (time.perf_counter() - h0) * 1e6 / K
            ev1.record()
            torch.cuda.synchronize()
            us = ev0.elapsed_time(ev1) * 1000.0 / K
            b1, f1, g1 = sh.greedy_band(), sh.greedy_fused_diag(), sh.greedy_diag()
            ex = f1["exact"] - f0["exact"] if form == "fused" else g1["fallbacks"] - g0["fallbacks"]
            res[form].append(us)
            if form == "fused":
                h, m = f1["hits"] - f0["hits"], f1["misses"] - f0["misses"]
            elif form in ("band", "adaptive"):
                h, m = b1["skips"] - b0["skips"], (b1["calls"] - b0["calls"]) - (b1["skips"] - b0["skips"])
            else:
                h, m = 0, 0
            cnt[form][0] += h
            cnt[form][1] += m
            print(f"{signal} rep {r} {form}: {us:.2f} us/tick (host enqueue {host_us:.2f}), hits {h} misses {m} exact {ex} of {K}",
                  flush=True)
    return {f: (statistics.median(res[f]), cnt[f][0], cnt[f][1]) for f in FORMS}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    signals = sys.argv[3].split(",") if len(sys.argv) > 3 else ["sinusoidals", "regular_steps", "perlin"]
    table = {s: run_signal(s, reps, K) for s in signals}
    print(f"\n{'signal':14s} " + " ".join(f"{f + ' us/tick':>15s} {'hit/miss':>10s}" for f in FORMS))
    for s, row in table.items():
        print(f"{s:14s} " + " ".join(f"{row[f][0]:15.2f} {row[f][1]:>5d}/{row[f][2]:<4d}" for f in FORMS))


if __name__ == "__main__":
    main()
