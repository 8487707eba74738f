"""Per-dispatch means of every counter of the rocprofv3 --pmc passes under SRC for the kernels whose
name contains KERNEL, into OUT (JSON; the pass CSVs are copied beside it as OUT_p<i>.csv).

    python tools/kernel_pmc_summary.py KERNEL SRC OUT.json
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def main():
    kern, src, out = sys.argv[1], sys.argv[2], sys.argv[3]
    acc = defaultdict(lambda: defaultdict(float))
    files = sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True))
    for i, f in enumerate(files):
        shutil.copy(f, out.replace(".json", f"_p{i + 1}.csv"))
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                acc[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    res = {"kernel": kern, "source": [os.path.basename(out.replace(".json", f"_p{i + 1}.csv")) for i in range(len(files))],
           "per_dispatch": {c: sum(v.values()) / len(v) for c, v in sorted(acc.items())},
           "dispatches": {c: len(v) for c, v in sorted(acc.items())}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["per_dispatch"]))


if __name__ == "__main__":
    main()
