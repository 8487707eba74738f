"""Copy a round's rocprofv3 outputs (gpurun_out/round, written by tools/pmc.sh passes) into
profiles/ under a round prefix and derive profiles/pmc_traffic.json: per kernel and shard size, the
HBM bytes per launch and the SQ instruction / stall counters.

    python tools/collect_profiles.py r02 [gpurun_out/round]

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE (KiB) is half the bytes of
wide coalesced streaming reads on gfx950 (doubled here; cross-checked against TCC_EA0_RDREQ x 128
B), WRITE_SIZE (KiB) is exact for 16-B-per-lane stores (cross-checked against TCC_EA0_WRREQ x 64
B).  Both count Infinity-Cache (MALL) hits, so while a working set fits the 256 MB MALL the figure
is memory-side traffic, not DRAM-only traffic; the TCC_EA0_*_DRAM counters are recorded beside it.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_step_window"


def per_dispatch(paths, kernel=KERNEL):
    """{counter: mean over dispatches of the per-dispatch sum} for kernels matching `kernel`."""
    acc = defaultdict(lambda: defaultdict(float))
    names = set()
    for path in paths:
        with open(path) as f:
            for r in csv.DictReader(f):
                if kernel not in r["Kernel_Name"]:
                    continue
                names.add(r["Kernel_Name"].split("(")[0])
                acc[r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {c: sum(v.values()) / len(v) for c, v in acc.items()}
    out["_dispatches"] = max((len(v) for v in acc.values()), default=0)
    out["_names"] = sorted(names)
    return out


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "round")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    with open(os.path.join(src, "bench.log")) as f:
        line = [ln for ln in f if ln.startswith("{")][-1]
    with open(os.path.join(dst, f"{tag}_bench.json"), "w") as f:
        f.write(line)
    for d in sorted(p for p in glob.glob(os.path.join(src, "stats_*")) if os.path.isdir(p)):  # WORKLOADS
        w = os.path.basename(d)[len("stats_"):]
        shutil.copy(os.path.join(d, "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_{w}_kernel_stats.csv"))
        with open(os.path.join(src, f"bench_{w}.log")) as f:
            lines = [ln for ln in f if ln.startswith("{")]
        if lines:
            with open(os.path.join(dst, f"{tag}_{w}_bench.json"), "w") as f:
                f.write(lines[-1])
    path = os.path.join(dst, "pmc_traffic.json")
    db = {}
    if os.path.exists(path):
        with open(path) as f:
            db = json.load(f)
    for d in sorted(p for p in glob.glob(os.path.join(src, "pmc_*")) if os.path.isdir(p)):
        houses = int(d.rsplit("_", 1)[1])
        csvs = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
        for i, p in enumerate(csvs):
            shutil.copy(p, os.path.join(dst, f"{tag}_pmc_{houses}_p{i + 1}.csv"))
        c = per_dispatch(csvs)
        fetch = c.get("FETCH_SIZE", 0.0) * 1024 * 2
        write = c.get("WRITE_SIZE", 0.0) * 1024
        rec = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in c.items()}
        rec.update({"hbm_bytes_per_launch": fetch + write, "read_bytes": fetch, "write_bytes": write,
                    "rdreq_x128_bytes": c.get("TCC_EA0_RDREQ", 0) * 128,
                    "wrreq_x64_bytes": c.get("TCC_EA0_WRREQ", 0) * 64,
                    "source": f"profiles/{tag}_pmc_{houses}_p*.csv (rocprofv3 --pmc over tools/kbench.py "
                              "--variants w32 --ticks 128: windows of 32 ticks)"})
        for name in c["_names"]:
            db.setdefault(name, {})[str(houses)] = rec
        print(houses, json.dumps({k: rec[k] for k in ("hbm_bytes_per_launch", "_dispatches", "_names")}))
    with open(path, "w") as f:
        json.dump(db, f, indent=1)


if __name__ == "__main__":
    main()
