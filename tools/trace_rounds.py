"""Per-dispatch durations from a rocprofv3 kernel trace (csv): the last
`--last` dispatches of the named kernels, in dispatch order (diagnostic)."""
import argparse
import csv

p = argparse.ArgumentParser()
p.add_argument("trace")
p.add_argument("--kernels", default="pb_route_kernel,pb_round_kernel,pt_round_kernel")
p.add_argument("--last", type=int, default=40)
a = p.parse_args()
names = a.kernels.split(",")
rows = []
with open(a.trace) as f:
    for r in csv.DictReader(f):
        k = r["Kernel_Name"]
        m = next((n for n in names if n in k), None)
        if m:
            rows.append((int(r["Start_Timestamp"]), m, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
rows.sort()
for _, m, us in rows[-a.last:]:
    print(f"{m:>18} {us:9.1f} us")
