"""Per-launch SQ / L2 counters of one kernel, launch by launch (for the
Plumtree round kernel: round by round), from one or more rocprofv3 --pmc
passes over the same deterministic run.

usage: python tools/pmc_rounds.py <kernel-substring> <pass1 counter_collection.csv> [<pass2 csv> ...]

Launches are matched across passes by their order.  Columns: busy cycles
(SQ_BUSY_CYCLES), wave-cycles per wave, the fraction of wave-cycles spent
waiting on anything (SQ_WAIT_ANY) / on instruction dependencies
(SQ_WAIT_INST_ANY), wave-instructions issued (VALU, SALU, vector memory read /
write, LDS), and the L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS))."""
import csv
import sys
from collections import OrderedDict


def launches(path, kname):
    per = OrderedDict()
    with open(path) as f:
        for row in csv.DictReader(f):
            if kname not in row["Kernel_Name"]:
                continue
            per.setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = float(row["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    kname, paths = sys.argv[1], sys.argv[2:]
    runs = [launches(p, kname) for p in paths]
    n = min(len(r) for r in runs)
    rows = []
    for i in range(n):
        d = {}
        for r in runs:
            d.update(r[i])
        rows.append(d)
    g = lambda d, k: d.get(k, float("nan"))  # noqa: E731
    print(f"{'#':>3} {'busy':>9} {'cyc/wave':>9} {'wait':>5} {'wdep':>5} {'VALU':>9} {'SALU':>9} {'VMrd':>8} "
          f"{'VMwr':>8} {'LDS':>8} {'L2hit':>6}")
    for i, d in enumerate(rows):
        wc, w = g(d, "SQ_WAVE_CYCLES"), g(d, "SQ_WAVES")
        hit, miss = g(d, "TCC_HIT_sum"), g(d, "TCC_MISS_sum")
        print(f"{i + 1:>3} {g(d, 'SQ_BUSY_CYCLES'):9.3g} {wc / w if w else float('nan'):9.0f} "
              f"{g(d, 'SQ_WAIT_ANY') / wc if wc else float('nan'):5.2f} "
              f"{g(d, 'SQ_WAIT_INST_ANY') / wc if wc else float('nan'):5.2f} "
              f"{g(d, 'SQ_INSTS_VALU'):9.3g} {g(d, 'SQ_INSTS_SALU'):9.3g} {g(d, 'SQ_INSTS_VMEM_RD'):8.3g} "
              f"{g(d, 'SQ_INSTS_VMEM_WR'):8.3g} {g(d, 'SQ_INSTS_LDS'):8.3g} "
              f"{hit / (hit + miss) if hit + miss else float('nan'):6.2f}")


if __name__ == "__main__":
    main()
