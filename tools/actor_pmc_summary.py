"""Summarise the k_actor counter passes of tools/pmc_actor.sh into profiles/<tag>_actor_pmc.json:
per launch and per 32-house tile (1M houses = 32,768 tiles), with the derived matrix-pipe and
VALU-issue fractions.  SQ_*_CYCLES counters are in units of 4 cycles (quad-cycles) on gfx950;
GRBM_GUI_ACTIVE is summed over the 8 XCDs.

    python tools/actor_pmc_summary.py TAG [gpurun_out/pmc_actor] [--copy]
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else os.path.join(ROOT, "gpurun_out", "pmc_actor")
    acc = defaultdict(lambda: defaultdict(float))
    files = sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True))
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "k_actor<" not in name and "k_actor(" not in name.replace("k_actor_pack", ""):
                continue
            if "k_actor_pack" in name:
                continue
            acc[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = {c: sum(v.values()) / len(v) for c, v in acc.items()}
    tiles = (1 << 20) // 32
    out = {"source": [os.path.relpath(f, ROOT) for f in files], "per_launch": per,
           "per_tile": {c: v / tiles for c, v in per.items()}}
    gui = per.get("GRBM_GUI_ACTIVE")
    if gui:
        cyc = gui / 8.0  # per XCD
        out["kernel_cycles"] = cyc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in per:
            out["mfma_busy_frac"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / cyc  # per SIMD
        if "SQ_INSTS_VALU" in per:
            out["valu_issue_frac"] = per["SQ_INSTS_VALU"] * 2.0 / 1024.0 / cyc  # 2 cycles per wave64 VALU issue
    dst = os.path.join(ROOT, "profiles", f"{tag}_actor_pmc.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    if "--copy" in sys.argv:
        for i, p in enumerate(files):
            shutil.copy(p, os.path.join(ROOT, "profiles", f"{tag}_actor_pmc_p{i + 1}.csv"))
    print(json.dumps({k: out[k] for k in ("kernel_cycles", "mfma_busy_frac", "valu_issue_frac") if k in out}))


if __name__ == "__main__":
    main()
