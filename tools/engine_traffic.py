"""Per-kernel HBM traffic of the non-headline engines (C2-C5) from rocprofv3:
a --kernel-trace --stats run (average launch duration per kernel) and two
separate --pmc passes, FETCH_SIZE and WRITE_SIZE (KiB per launch; the
MI355X_MICROARCH.md HBM recipe: they do not fit one pass; FETCH_SIZE
undercounts wide coalesced streaming reads by half on gfx950, so the doubled
read side is given as the upper bound).

usage: python tools/engine_traffic.py <stats_dir> <fetch_dir> <write_dir> [--out f.json]
"""
import argparse
import collections
import csv
import json
import os


def pmc(d, counter):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            out[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return out


def stats(d):
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        out[r["Name"]] = dict(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3,
                              total_ms=float(r["TotalDurationNs"]) / 1e6, pct=float(r["Percentage"]))
    return out


def short(name):
    return name.replace("psim::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("stats_dir")
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--top", type=int, default=14)
    p.add_argument("--out")
    a = p.parse_args()
    st = stats(a.stats_dir)
    f, w = pmc(a.fetch_dir, "FETCH_SIZE"), pmc(a.write_dir, "WRITE_SIZE")
    rows = []
    for name, s in sorted(st.items(), key=lambda kv: -kv[1]["total_ms"])[: a.top]:
        fs, ws = f.get(name, []), w.get(name, [])
        fb = sum(fs) / len(fs) if fs else None
        wb = sum(ws) / len(ws) if ws else None
        r = dict(kernel=short(name), calls=s["calls"], avg_us=round(s["avg_us"], 2), total_ms=round(s["total_ms"], 3),
                 pct=round(s["pct"], 2), fetch_bytes_per_launch=fb, write_bytes_per_launch=wb)
        if fb is not None and wb is not None and s["avg_us"] > 0:
            r["hbm_GBps_measured"] = round((fb + wb) / (s["avg_us"] * 1e3), 1)
            r["hbm_GBps_read_doubled"] = round((2 * fb + wb) / (s["avg_us"] * 1e3), 1)
        rows.append(r)
    print(json.dumps(rows, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)
            fh.write("\n")


if __name__ == "__main__":
    main()
