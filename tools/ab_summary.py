"""ms_per_step (timed and sustained) of bench A/B logs: python tools/ab_summary.py gpurun_out b_new b_old"""
import glob
import json
import os
import sys

d = sys.argv[1]
for pre in sys.argv[2:]:
    rows = []
    for f in sorted(glob.glob(os.path.join(d, pre + "_*.log"))):
        for line in open(f):
            if line.startswith("{"):
                j = json.loads(line)
                rows.append((round(j["ms_per_step"], 4), round(j.get("sustained", {}).get("ms_per_step", 0), 4)))
    print(pre, rows)
