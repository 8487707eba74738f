"""Split a rocprofv3 kernel trace's launches of one kernel by size class (the bench runs the benched
kernel at 1M houses and, for roofline.above_mall, at 16M in the same process, so the --stats average
mixes the two).  Writes {class: {launches, avg_us, min_us, max_us}}.

    python tools/split_stats.py TRACE_CSV KERNEL_SUBSTRING THRESHOLD_US OUT_JSON
"""
import csv
import json
import statistics
import sys


def main():
    trace, kern, thr, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(trace))
         if kern in r["Kernel_Name"]]
    res = {"kernel": kern, "source": trace, "threshold_us": thr}
    for name, xs in (("below", [x for x in d if x < thr]), ("above", [x for x in d if x >= thr])):
        if xs:
            res[name] = {"launches": len(xs), "avg_us": statistics.mean(xs), "min_us": min(xs), "max_us": max(xs)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
