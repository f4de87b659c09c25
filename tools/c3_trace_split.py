"""C3 kernel durations by phase from a rocprofv3 kernel trace of
tools/c3_wall.py (diagnostic): the join-wave build, the settle rounds and the
churn rounds have very different loads, so an average over every call (the
--stats line) says nothing about imbalance inside one round.  Prints, per
kernel, the average and max duration over the LAST `churn` calls (the churn
rounds c3_wall.py times) and over all calls.

usage: python tools/c3_trace_split.py gpurun_out/c3prof [churn=30]"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    churn = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    for k in ("sc_process", "pd_process", "sc_scatter", "pd_scatter"):
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
                if ("::" + k + "(") in r["Kernel_Name"]]
        if not durs:
            continue
        last = durs[-churn:]
        out[k] = {"calls": len(durs), "all_avg_us": round(sum(durs) / len(durs), 1), "all_max_us": round(max(durs), 1),
                  "churn_avg_us": round(sum(last) / len(last), 1), "churn_max_us": round(max(last), 1),
                  "churn_max_over_avg": round(max(last) / (sum(last) / len(last)), 2),
                  "churn_us": [round(x, 1) for x in last]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
