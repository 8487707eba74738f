"""Copy a round's rocprofv3 outputs (gpurun_out/round, written by tools/profile_round.sh) into
profiles/ under a round prefix and derive profiles/pmc_traffic.json (HBM bytes per k_step launch).

    python tools/collect_profiles.py r01 [gpurun_out/round]

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE (KiB) is half the bytes of
wide coalesced streaming reads on gfx950 (doubled here; cross-checked against TCC_EA0_RDREQ x 128
B), WRITE_SIZE (KiB) is exact for 16-B-per-lane stores (cross-checked against TCC_EA0_WRREQ x 64
B).  Both count Infinity-Cache (MALL) hits, so at 1M houses (~94 MB/tick, MALL-resident) the
figure is memory-side traffic, not DRAM-only traffic.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, kernel="k_step"):
    """{counter: mean over dispatches of the per-dispatch sum} for kernels matching `kernel`."""
    acc = defaultdict(lambda: defaultdict(float))
    grid = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
    out = {c: sum(v.values()) / len(v) for c, v in acc.items()}
    out["_dispatches"] = max((len(v) for v in acc.values()), default=0)
    out["_grid"] = sorted(set(grid.values()))
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
    bench = json.loads(line)
    houses = bench["config"]["houses_per_gpu"]
    c = {}
    for d in ("pmc_fetch", "pmc_write", "pmc_dram"):
        p = os.path.join(src, d, "run_counter_collection.csv")
        shutil.copy(p, os.path.join(dst, f"{tag}_{d}.csv"))
        c.update(per_dispatch(p))
    fetch = c["FETCH_SIZE"] * 1024 * 2
    write = c["WRITE_SIZE"] * 1024
    rec = {
        "hbm_bytes_per_launch": fetch + write,
        "read_bytes": fetch, "write_bytes": write,
        "FETCH_SIZE_KiB": c["FETCH_SIZE"], "WRITE_SIZE_KiB": c["WRITE_SIZE"],
        "TCC_EA0_RDREQ": c.get("TCC_EA0_RDREQ"), "TCC_EA0_WRREQ_DRAM": c.get("TCC_EA0_WRREQ_DRAM"),
        "rdreq_x128_bytes": c.get("TCC_EA0_RDREQ", 0) * 128,
        "wrreq_x64_bytes": c.get("TCC_EA0_WRREQ_DRAM", 0) * 64,
        "bytes_per_house_step": (fetch + write) / houses,
        "dispatches": c["_dispatches"], "grid": c["_grid"],
        "kernel": "mdr::k_step_t<2,false,true,RANDOM,RANDOM>",
        "source": f"profiles/{tag}_pmc_*.csv (rocprofv3 --pmc, one counter group per pass)",
    }
    path = os.path.join(dst, "pmc_traffic.json")
    db = {}
    if os.path.exists(path):
        with open(path) as f:
            db = json.load(f)
    db[str(houses)] = rec
    with open(path, "w") as f:
        json.dump(db, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
