"""Per-call critical path of a rollout call from a rocprofv3 kernel + HIP API trace (csv): the
kernels of the last calls in stream order with their durations and the gaps before them, and the
host API calls that issued them.  A call starts at each k_count_window launch.

    python tools/trace_calls.py <dir with run_kernel_trace.csv and run_hip_api_trace.csv> [calls]
"""
import csv
import os
import sys


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "mdr::"):
        n = n.replace(p, "")
    return n[:48]


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    kern = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))), key=lambda k: int(k["Start_Timestamp"]))
    api = list(csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))))
    by_corr = {a["Correlation_Id"]: a for a in api}
    starts = [i for i, k in enumerate(kern) if "k_count_window" in k["Kernel_Name"]]
    calls = [(starts[j], starts[j + 1] if j + 1 < len(starts) else len(kern)) for j in range(len(starts))]
    spans = []
    for a, b in calls[-last - 1:-1]:
        t0 = int(kern[a]["Start_Timestamp"])
        a_api = by_corr.get(kern[a]["Correlation_Id"])
        print(f"--- call at kernel {a}: first launch API began {(t0 - int(a_api['Start_Timestamp'])) / 1e3:.1f} us before the count started" if a_api else "--- call")
        prev_end = t0
        for k in kern[a:b]:
            s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
            print(f"  +{(s - t0) / 1e3:7.1f} us  gap {(s - prev_end) / 1e3:6.1f}  dur {(e - s) / 1e3:6.1f}  {short(k['Kernel_Name'])}")
            prev_end = e
        spans.append((prev_end - t0) / 1e3)
        print(f"  first kernel start -> last kernel end: {(prev_end - t0) / 1e3:.1f} us")
    if spans:
        print("spans:", " ".join(f"{x:.1f}" for x in spans))


if __name__ == "__main__":
    main()
