"""Summarise rocprofv3 --pmc CSVs: per-kernel mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?")
            k = k.split("(")[0][:60]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    if "k_step" not in k and "probe" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        # per-dispatch values are summed over dimensions already by rocprofv3; average dispatches
        print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
