"""Per-launch HBM traffic of the Plumtree round kernel from rocprofv3 PMC passes.

Collected as MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7 prescribe:
two separate --pmc passes (FETCH_SIZE, WRITE_SIZE; they do not fit one
pass), units KiB (hbm bytes = (FETCH_SIZE + WRITE_SIZE) * 1024).  The gfx950
caveat: FETCH_SIZE counts exactly half the bytes of WIDE coalesced streaming
reads; this kernel's reads are mostly narrow/scattered, so the raw value is
reported and the doubled read side is given as an upper bound.

usage: python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
          --n 10000000 --peers 5 --rounds-per-step 16 --steps 3 [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import json
import os


def load(d, counter, kernel):
    path = os.path.join(d, "run_counter_collection.csv")
    rows = [r for r in csv.DictReader(open(path))
            if ("::" + kernel + "<") in r["Kernel_Name"] or ("::" + kernel + "(") in r["Kernel_Name"]]
    return [float(r["Counter_Value"]) * 1024.0 for r in rows if r["Counter_Name"] == counter]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--n", type=int, required=True)
    p.add_argument("--peers", type=int, required=True)
    p.add_argument("--rounds-per-step", type=int, required=True)
    p.add_argument("--steps", type=int, required=True, help="steps incl. warmup in the profiled run")
    p.add_argument("--kernel", default="pt_round_ell_kernel",
                   help="the round kernel bench.py runs (ELL rows: pt_round_ell_kernel; CSR: pt_round_kernel)")
    p.add_argument("--out", default=None)
    p.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "partisan_amd", "libpsim.so"),
                   help="the libpsim.so the profiled run loaded: bench.py reports the traffic only for this build")
    p.add_argument("--source", default=None, help="where the raw rocprofv3 outputs are kept (profiles/...)")
    a = p.parse_args()
    import hashlib
    with open(a.lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    f = load(a.fetch_dir, "FETCH_SIZE", a.kernel)
    w = load(a.write_dir, "WRITE_SIZE", a.kernel)
    counted = a.rounds_per_step * a.steps
    fetch = sum(f) / counted
    write = sum(w) / counted
    # per round of a step: launch i of every step (the run repeats the same
    # deterministic flood, so launch k * rounds_per_step + i is round i + 1)
    per_round = []
    if len(f) == counted and len(w) == counted:
        R = a.rounds_per_step
        for i in range(R):
            per_round.append({"round": i + 1, "fetch": sum(f[k * R + i] for k in range(a.steps)) / a.steps,
                              "write": sum(w[k * R + i] for k in range(a.steps)) / a.steps})
    out = {
        "n": a.n, "peers": a.peers, "kernel": a.kernel,
        "launches_profiled": len(f), "counted_launches": counted,
        "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "hbm_bytes_per_launch_read_doubled": 2 * fetch + write,
        "per_round": per_round,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB*1024, "
                  "summed over all launches of the kernel / counted rounds",
        "lib_sha256": lib_sha,
        "source": a.source,
    }
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)
            fh.write("\n")


if __name__ == "__main__":
    main()
