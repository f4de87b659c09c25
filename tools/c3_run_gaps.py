"""Timeline of the last R C3 rounds under rocprofv3 --kernel-trace
--memory-copy-trace (tools/c3_wall.py ... run): device time per kernel /
copy kind and the idle gaps between consecutive operations, per round.

usage: python tools/c3_run_gaps.py <dir with run_kernel_trace.csv> [R]"""
import collections
import csv
import json
import re
import os
import sys


def main():
    d = sys.argv[1]
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ops = []
    with open(os.path.join(d, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            n = re.sub(r"\((psim::|unsigned).*", "", n).split("::")[-1][:40]
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        with open(p) as f:
            for r in csv.DictReader(f):
                ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"]))
    ops.sort()
    ends = [i for i, o in enumerate(ops) if o[2].startswith("pd_process")]
    lo, hi = ends[-R - 1], ends[-1]
    win = ops[lo + 1:hi + 1]
    busy = collections.Counter()
    cnt = collections.Counter()
    idle = 0
    t = ops[lo][1]
    for s, e, n in win:
        busy[n] += e - s
        cnt[n] += 1
        if s > t:
            idle += s - t
        t = max(t, e)
    span = ops[hi][1] - ops[lo][1]
    out = {"rounds": R, "span_us_per_round": round(span / R / 1e3, 2), "idle_us_per_round": round(idle / R / 1e3, 2),
           "ops_per_round": round(len(win) / R, 1),
           "busy_us_per_round": {k: round(v / R / 1e3, 2) for k, v in busy.most_common()},
           "calls_per_round": {k: round(v / R, 2) for k, v in cnt.most_common()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
