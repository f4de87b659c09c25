"""Per-step timeline of a bench.py run under rocprofv3 --kernel-trace
--memory-copy-trace: for each step (pt_origin_kernel .. the last round
kernel before the next origin) the span, the kernels' busy time, the copies
and the idle gaps between consecutive operations.

usage: python tools/trace_gaps.py <dir with run_kernel_trace.csv>"""
import csv
import os
import sys


def short(name):
    for k in ("pt_round_ell_kernel", "pt_round_kernel", "pt_origin_kernel", "pt_prep_kernel", "fillBuffer", "copyBuffer"):
        if k in name:
            return k
    return name[:40]


def main():
    d = sys.argv[1]
    ops = []
    with open(os.path.join(d, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        with open(p) as f:
            for r in csv.DictReader(f):
                ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"][12:]))
    ops.sort()
    starts = [i for i, o in enumerate(ops) if "pt_origin_kernel" in o[2]]
    for si, i in enumerate(starts[:-1] if len(starts) > 1 else starts):
        j = starts[si + 1] if si + 1 < len(starts) else len(ops)
        seg = ops[i:j]
        # the step ends at its last round kernel
        last = max(k for k, o in enumerate(seg) if "round" in o[2])
        seg = seg[:last + 1]
        span = (seg[-1][1] - seg[0][0]) / 1e3
        busy = sum(o[1] - o[0] for o in seg if not o[2].startswith("copy")) / 1e3
        gaps = [(seg[k + 1][0] - seg[k][1]) / 1e3 for k in range(len(seg) - 1)]
        big = sorted(((g, seg[k][2], seg[k + 1][2]) for k, g in enumerate(gaps)), reverse=True)[:4]
        print(f"step {si}: span {span:.1f} us, kernels {busy:.1f} us, ops {len(seg)}, gaps sum {sum(gaps):.1f} us, "
              f"largest {[(round(g, 1), a, b) for g, a, b in big]}")
        if si + 1 < len(starts):   # between steps: the step's last operation (its stats copy) to the next origin
            tail = ops[i:j]
            t_end = max(o[1] for o in tail)
            after = [o for o in tail if o[0] >= seg[-1][1]]
            print(f"   between steps: {len(after)} ops after the last round "
                  f"({', '.join(f'{a[2]} {(a[1] - a[0]) / 1e3:.1f} us' for a in after)}), "
                  f"device idle until the next origin {(ops[j][0] - t_end) / 1e3:.1f} us, "
                  f"last round end to next origin {(ops[j][0] - seg[-1][1]) / 1e3:.1f} us")
        if si == 0:
            for o in seg:
                print(f"   {(o[0] - seg[0][0]) / 1e3:9.1f} {(o[1] - o[0]) / 1e3:8.1f}  {o[2]}")


if __name__ == "__main__":
    main()
