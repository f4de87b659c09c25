"""Per-launch means of rocprofv3 --pmc counters for one kernel.

usage: python tools/pmc_summary.py <counter_collection.csv> <kernel-substring> [units-per-launch] [skip]

Prints every counter's mean over the kernel's launches (after skipping the
first `skip`), and, given the units one launch processes (C5: vertices of a
round), the VALU / SALU / LDS wave-instructions per unit and the issue bound
they imply: instructions x units / (256 CUs x 4 SIMDs) x 4 cycles per
instruction issue slot, at 2.4 GHz (MI355X_MICROARCH.md)."""
import csv
import sys
from collections import defaultdict


def main():
    path, kname = sys.argv[1], sys.argv[2]
    units = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    per = defaultdict(dict)            # dispatch id -> counter -> value
    with open(path) as f:
        for row in csv.DictReader(f):
            if kname not in row["Kernel_Name"]:
                continue
            per[int(row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
    ids = sorted(per)[skip:]
    if not ids:
        raise SystemExit(f"no launches of {kname} in {path}")
    names = sorted({c for i in ids for c in per[i]})
    mean = {c: sum(per[i].get(c, 0.0) for i in ids) / len(ids) for c in names}
    print(f"{kname}: {len(ids)} launches (first {skip} skipped), per launch:")
    for c in names:
        print(f"  {c:<24} {mean[c]:.4g}")
    if units:
        v, s = mean.get("SQ_INSTS_VALU", 0.0) / units, mean.get("SQ_INSTS_SALU", 0.0) / units
        simds, clk = 256 * 4, 2.4e9
        print(f"per unit: VALU {v:.0f}, SALU {s:.0f}, LDS {mean.get('SQ_INSTS_LDS', 0.0) / units:.0f} wave-instructions")
        for nm, x in (("VALU", v), ("SALU", s)):
            print(f"  {nm} issue bound: {x * units / simds * 4 / clk * 1e3:.3f} ms per launch")
        if "SQ_WAVE_CYCLES" in mean and mean["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if c in mean:
                    print(f"  {c} / SQ_WAVE_CYCLES = {mean[c] / mean['SQ_WAVE_CYCLES']:.2f}")


if __name__ == "__main__":
    main()
