"""s_memrealtime split of k_count_window: build the variant library with the
timestamps (python marl-demandresponse_amd/build_ext.py --variant cwt MDR_COUNT_TIMING), then

    MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwt.so python tools/count_timing.py [--ticks 20]

Per launch (1M houses, random actions, the first window of a rollout as mdr_rollout_begin issues it):
the 100 MHz clock of every block at entry (t0), after its state loads were consumed (t1), after
its shard flush (t2) and after its ticket (t3; the last block: after its P-only reduce)."""
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
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--waves", type=int, default=16, help="waves per count block (the library's MDR_COUNT_WAVES)")
    a = ap.parse_args()
    import torch

    from bench import env_props
    from mdr_amd import _lib as L
    from mdr_amd.environment import Environment

    env = Environment(env_props(a.houses), device="cuda:0", rng=random.Random(1), population="synthetic", seed=5)
    sh = env.shard
    lib = L.load()
    fn = lib.mdr_count_timing
    fn.argtypes = [C.c_void_p, C.c_int]
    hpb = 128 * a.waves  # houses per block
    nb = (a.houses + hpb - 1) // hpb
    buf = np.zeros(nb * 4, np.uint64)
    rows = []
    for r in range(a.reps + 2):
        torch.cuda.synchronize()
        sh.rollout_begin(a.ticks, 0, None, 0, L.ACT_RANDOM)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, nb) == 0
        t = buf.reshape(nb, 4).astype(np.int64)
        t = (t - t[:, 0].min()) * 10  # ns
        last = int(np.argmax(t[:, 3]))
        rows.append([t[:, 0].max(), np.median(t[:, 1] - t[:, 0]), np.median(t[:, 2] - t[:, 1]),
                     np.median(t[:, 3] - t[:, 2]), t[last, 3] - t[last, 2], t[:, 2].max(), t[:, 3].max()])
    rows = np.array(rows[2:], np.float64) / 1e3
    names = ["dispatch spread (last block start)", "load (median t1-t0)", "FSM + stores + flush (median t2-t1)",
             "ticket (median t3-t2)", "last block's ticket + reduce", "last flush done", "kernel span (last t3)"]
    print(f"k_count_window, {a.houses} houses, {a.ticks} ticks, {nb} blocks: us (median over {a.reps} launches)")
    for i, nm in enumerate(names):
        print(f"  {nm:40s} {np.median(rows[:, i]):7.2f}  (min {rows[:, i].min():.2f}, max {rows[:, i].max():.2f})")


if __name__ == "__main__":
    main()
