"""Sum the HBM bytes of one greedy + step tick (config C3) from the rocprofv3 counter passes of
tools/pmc_greedy.sh: per kernel the mean per-dispatch FETCH_SIZE (x 2: gfx950 counts half the bytes of
wide coalesced reads, MI355X_MICROARCH.md) + WRITE_SIZE, summed over the tick's three kernels, and
recorded in profiles/pmc_traffic.json under the greedy line's kernel name at 1,048,576 houses
(round 5: the band's two launches after the step, tools/pmc_greedy.sh).

    python tools/greedy_pmc_summary.py TAG gpurun_out/pmc_greedy
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ["k_step_pipe<2, 0, 0, 1>", "k_gq_binsc", "k_gq_finish"]
LINE_KERNEL = ("greedy tick: histogram select (k_gq_binsc, k_gq_finish; codes, superbin and predicted-band "
               "bin counts from the previous k_step_pipe's epilogue) + k_step_pipe")


def main():
    tag, src = sys.argv[1], sys.argv[2]
    per = {k: defaultdict(lambda: defaultdict(float)) for k in KERNELS}
    files = sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True))
    for i, f in enumerate(files):
        shutil.copy(f, os.path.join(ROOT, "profiles", f"{tag}_greedy_pmc_p{i + 1}.csv"))
        for r in csv.DictReader(open(f)):
            for k in KERNELS:
                if k in r["Kernel_Name"]:
                    per[k][r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    total = 0.0
    for k in KERNELS:
        c = {n: sum(v.values()) / len(v) for n, v in per[k].items() if v}
        b = c.get("FETCH_SIZE", 0.0) * 1024 * 2 + c.get("WRITE_SIZE", 0.0) * 1024
        out[k] = {"hbm_bytes_per_launch": b, **{n: round(x, 1) for n, x in c.items()}}
        total += b
    rec = {"hbm_bytes_per_launch": total, "per_kernel": out,
           "source": f"profiles/{tag}_greedy_pmc_p*.csv (rocprofv3 --pmc over bench.py --workload greedy)"}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(path)) if os.path.exists(path) else {}
    db.setdefault(LINE_KERNEL, {})["1048576"] = rec
    json.dump(db, open(path, "w"), indent=1)
    print(json.dumps({"tick_bytes": total, **{k: v["hbm_bytes_per_launch"] for k, v in out.items()}}))


if __name__ == "__main__":
    main()
