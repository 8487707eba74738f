"""The fused greedy decision's phases (k_gq_decide2 phase stamps, mdr_greedy_fused_stamps): C3's loop at
1M houses, then single-tick mdr_greedy_rollout calls with the stamps on; per phase, microseconds from the
kernel's first block entry (median over the calls): every block's phase ends (median / max over blocks),
the deciding block's and block 0's.

    python tools/greedy_fused_probe.py [--houses 1048576] [--calls 20]
"""
import argparse
import ctypes as C
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd"), os.path.join(ROOT, "tests")]
import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=20)
    a = ap.parse_args()
    import torch

    import golden_util as gu
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": a.houses,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(53), population="synthetic", seed=53)
    sh = env.shard
    lib = sh.lib
    sh.set_option("gq_fused", 1)
    env.greedy_rollout(30)
    L.check(lib.mdr_greedy_fused_stamps(sh.ctx, 1, None), "stamps on")
    names = ["entry", "super_scan", "A_prefix", "window", "gather", "rank", "ticket", "decided", "next_map", "exit",
             "lastflag", "apre_done", "d_loaded", "d_cross", "d_walk", "d_counts", "sup_loaded", "A_loaded", "g_counts", "g_loaded", "g_ranked", "-", "-", "t0_ranked", "t0_bar", "-", "-", "scan_summed", "scan_blockscan", "scan_first", "scan_end"]
    per = {k: [] for k in names}
    lastb, blk0 = {k: [] for k in names}, {k: [] for k in names}
    for _ in range(a.calls):
        env.greedy_rollout(1)
        torch.cuda.synchronize()
        buf = (C.c_uint64 * (256 * 32))()
        L.check(lib.mdr_greedy_fused_stamps(sh.ctx, 1, buf), "stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 32).astype(np.int64)
        t0 = st[:, 0].min()
        for k, nm in enumerate(names):
            if nm in ("lastflag", "-"):
                continue
            col = st[:, k]
            ok = col > 0
            if ok.any():
                per[nm].append((np.median(col[ok] - t0) / 100.0, (col[ok] - t0).max() / 100.0))
        print("gather npair/total (block 0):", st[0, 21], st[0, 22])
        li = int(np.nonzero(st[:, 10] == 1)[0][0]) if (st[:, 10] == 1).any() else -1
        for k, nm in enumerate(names):
            if li >= 0 and st[li, k] > 0:
                lastb[nm].append((st[li, k] - t0) / 100.0)
            if st[0, k] > 0:
                blk0[nm].append((st[0, k] - t0) / 100.0)
        buf2 = (C.c_uint64 * (256 * 32))()
        L.check(lib.mdr_greedy_fused_stamps(sh.ctx, 0, None), "reset")
        L.check(lib.mdr_greedy_fused_stamps(sh.ctx, 1, None), "on")
    print("fused diag", sh.greedy_fused_diag())
    print(f"{'phase':12s} {'all blocks med':>14s} {'max':>8s} {'last block':>11s} {'block 0':>8s}   (us from the first entry)")
    for nm in names:
        if per[nm]:
            m = np.median([x[0] for x in per[nm]]), np.median([x[1] for x in per[nm]])
            lb = np.median(lastb[nm]) if lastb[nm] else float("nan")
            b0 = np.median(blk0[nm]) if blk0[nm] else float("nan")
            print(f"{nm:12s} {m[0]:14.2f} {m[1]:8.2f} {lb:11.2f} {b0:8.2f}")


if __name__ == "__main__":
    main()
