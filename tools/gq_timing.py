"""s_memrealtime split of the greedy select launch (k_gq_select1): build the variant library with the
timestamps (python marl-demandresponse_amd/build_ext.py --variant gqt MDR_GQ_TIMING), then

    MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gqt.so python tools/gq_timing.py

Config C3 (1M houses, greedy + step per tick); after each greedy call the 100 MHz clock of block 0 at
entry, window loaded, ranked, crossing found, walk done, end, and of block 1 at entry and map done."""
import argparse
import ctypes as C
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-demandresponse_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--houses", type=int, default=1 << 20)
    ap.add_argument("--ticks", type=int, default=30)
    a = ap.parse_args()
    import torch

    from bench import env_props
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    env = Environment(env_props(a.houses), device="cuda:0", rng=random.Random(1), population="synthetic", seed=5)
    lib = L.load()
    fn = lib.mdr_gq_timing
    fn.argtypes = [C.c_void_p]
    buf = np.zeros(16, np.uint64)
    n = env.n_local
    act = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rew = torch.empty(n, dtype=torch.float64, device="cuda:0")
    rows = []
    for t in range(a.ticks + 3):
        env.greedy_actions(out=act)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data) == 0
        ts = buf.astype(np.int64)
        base = ts[[0, 6]].min()
        clk = [(ts[8 + 5] - ts[8]) / max(1, ts[5] - ts[0]) * 0.1, (ts[8 + 7] - ts[8 + 6]) / max(1, ts[7] - ts[6]) * 0.1]
        rows.append(list((ts[:8] - base) * 10) + clk)  # ns, GHz
        env.step_tensor(act, rewards=rew, ctrl="greedy_keys")
    r = np.array(rows[3:], np.float64) / 1e3
    names = ["block 0 entry", "window loaded", "ranked", "crossing found", "walk done", "block 0 end",
             "block 1 entry", "block 1 map done"]
    print(f"k_gq_select1, {a.houses} houses: us after the earlier block's entry (median over {a.ticks} calls)")
    for i, nm in enumerate(names):
        print(f"  {nm:22s} {np.median(r[:, i]):7.2f}  (min {r[:, i].min():.2f}, max {r[:, i].max():.2f})")
    r2 = np.array(rows[3:], np.float64)
    for i, nm in enumerate(["block 0 shader clock", "block 1 shader clock"]):
        print(f"  {nm:22s} {np.median(r2[:, 8 + i]):7.2f} GHz  (min {r2[:, 8 + i].min():.2f}, max {r2[:, 8 + i].max():.2f})")


if __name__ == "__main__":
    main()
