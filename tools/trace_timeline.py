"""Print a rocprofv3 kernel trace as a timeline (start offset, duration, gap to the previous kernel).

    python3 tools/trace_timeline.py run_kernel_trace.csv [--last N] [--match NAME]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--first", type=int, default=0)
ap.add_argument("--count", type=int, default=60)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[a.first:a.first + a.count]
t0, prev = int(rows[0]["Start_Timestamp"]), None
for i, r in enumerate(rows):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{a.first + i:4d} {r['Kernel_Name'][:44]:44s} t={(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:7.1f}")
    prev = e
