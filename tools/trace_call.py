"""The timed 20-step call in a rocprofv3 kernel + HIP API trace of `bench.py --steps 20`: for each of
the last rollout calls (a k_count_window launch followed by its step kernel), the API time of the
count's launch, when the count kernel started after that launch was issued, both kernels' durations,
the gap between them and when the synchronisation returned.  Usage:
python tools/trace_call.py <dir with run_kernel_trace.csv and run_hip_api_trace.csv> [calls]"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    kern = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    api = list(csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))))
    by_corr = {a["Correlation_Id"]: a for a in api}
    syncs = sorted((int(a["Start_Timestamp"]), int(a["End_Timestamp"])) for a in api
                   if a["Function"] in ("hipStreamSynchronize", "hipDeviceSynchronize", "hipEventSynchronize"))
    kern.sort(key=lambda k: int(k["Start_Timestamp"]))
    # the rollout calls' first windows: a count followed directly by the KA step kernel
    calls = [i for i, k in enumerate(kern) if "k_count_window" in k["Kernel_Name"] and i + 1 < len(kern)
             and "k_step_window" in kern[i + 1]["Kernel_Name"]]
    for i in calls[-last:]:
        c, s = kern[i], kern[i + 1] if i + 1 < len(kern) else None
        a = by_corr.get(c["Correlation_Id"])
        cs, ce = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
        line = f"count launch API {(int(a['End_Timestamp']) - int(a['Start_Timestamp'])) / 1e3:6.1f} us, " \
               f"kernel start {(cs - int(a['Start_Timestamp'])) / 1e3:6.1f} us after the API call began; " if a else ""
        line += f"count {(ce - cs) / 1e3:5.1f} us"
        if s is not None:
            ss, se = int(s["Start_Timestamp"]), int(s["End_Timestamp"])
            sa = by_corr.get(s["Correlation_Id"])
            line += f"; gap {(ss - ce) / 1e3:4.1f}; {s['Kernel_Name'].split('(')[0][-40:]} {(se - ss) / 1e3:5.1f} us"
            if sa:
                line += f" (its launch API began {(int(sa['Start_Timestamp']) - int(a['Start_Timestamp'])) / 1e3:5.1f} us after the count's)" if a else ""
            after = [e for st, e in syncs if e >= se]
            if after:
                line += f"; sync returned {(after[0] - se) / 1e3:4.1f} us after the step ended"
        print(line)


if __name__ == "__main__":
    main()
