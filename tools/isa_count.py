"""Static instruction mix of one kernel in a -save-temps .s (hipcc
--offload-arch=gfx950 -save-temps): instructions by class, the most common
opcodes, v_readlane / v_writelane (SGPR spill traffic), 64-bit address math,
and per basic block (label) counts so the hot loop can be located.

--loops: the same per loop (LLVM's "Loop: Header=... Depth=" block notes),
innermost loop of each block, with its memory operations -- which candidate
or arrival loop holds the spill reloads.

usage: python tools/isa_count.py <file.s> <kernel-substring> [--blocks] [--loops]"""
import re
import sys
from collections import Counter


def body(path, name):
    s = open(path).read()
    m = re.search(r"^(\S*" + re.escape(name) + r"\S*):[^\n]*\n", s, re.M)
    if not m:
        raise SystemExit(f"no kernel matching {name}")
    i = m.end()
    j = s.index(".Lfunc_end", i)
    return m.group(1), s[i:j]


def cls(op):
    if op.startswith("s_"):
        return "SALU" if not op.startswith(("s_load", "s_buffer_load", "s_waitcnt", "s_barrier", "s_cbranch",
                                            "s_branch", "s_endpgm", "s_nop", "s_sleep")) else \
            ("SMEM" if "load" in op else "control")
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    fname, b = body(path, name)
    blocks, cur = [], ("entry", [])
    for raw in b.split("\n"):
        line = raw.split(";")[0].strip()
        if not line or line.startswith("."):
            if raw.strip().startswith(".LBB"):
                pass
            continue
        if line.endswith(":"):
            blocks.append(cur)
            cur = (line[:-1], [])
            continue
        cur[1].append(line)
    blocks.append(cur)
    ins = [l for _, bl in blocks for l in bl]
    ops = Counter(l.split()[0] for l in ins)
    c = Counter()
    for op, k in ops.items():
        c[cls(op)] += k
    print(f"{fname}: {len(ins)} instructions")
    print("  by class:", dict(c))
    print("  v_readlane / v_writelane:", sum(k for op, k in ops.items() if "readlane" in op or "writelane" in op),
          " scratch:", sum(k for op, k in ops.items() if op.startswith("scratch_")))
    print("  64-bit adds (v_lshl_add_u64 / v_add_co / v_addc):",
          sum(k for op, k in ops.items() if op in ("v_lshl_add_u64", "v_add_co_u32_e32", "v_add_co_u32_e64",
                                                   "v_addc_co_u32_e32", "v_addc_co_u32_e64", "v_add_u64",
                                                   "v_lshlrev_b64", "v_mad_u64_u32")))
    print("  top opcodes:", ops.most_common(30))
    if "--loops" in sys.argv:
        per, mem, cur = {}, {}, (0, "-")
        for raw in b.split("\n"):
            st = raw.strip()
            if (raw[:1] not in (" ", "\t") and st.endswith(":")) or st.startswith("; %bb") or \
                    (st.startswith(".LBB") and ":" in st):
                import re
                m = re.search(r"Loop: Header=(\S+) Depth=(\d+)", raw)
                cur = (int(m.group(2)), m.group(1)) if m else (0, "-")
                continue
            line = raw.split(";")[0].strip()
            if not line or line.startswith(".") or line.endswith(":"):
                continue
            op = line.split()[0]
            per.setdefault(cur, Counter())[cls(op)] += 1
            if cls(op) in ("VMEM", "LDS") or "readlane" in op or "writelane" in op:
                mem.setdefault(cur, Counter())[op] += 1
        for k in sorted(per, key=lambda k: (k[0], k[1])):
            print(f"  depth {k[0]} {k[1]:>12} {dict(per[k])} {dict(mem.get(k, {}))}")
    if "--blocks" in sys.argv:
        for lab, bl in blocks:
            bc = Counter(cls(l.split()[0]) for l in bl)
            print(f"  {lab:>12} {len(bl):5d} {dict(bc)}")


if __name__ == "__main__":
    main()
