"""Static instructions of one kernel attributed to source lines (diagnostic):
compile with line tables (hipcc -O3 -gline-tables-only --cuda-device-only -S)
and every instruction after a `.loc <file> <line>` directive counts for that
line.  Prints the top lines by VALU / SALU count, optionally only inside the
loop whose header label is given (instructions from the label to the loop's
back-edge branch to it).

usage: python tools/isa_lines.py <.s> <kernel symbol> [--file plumtree.hip] [--loop .LBB30_1430] [--top 40]"""
import argparse
import collections
import re


def main():
    p = argparse.ArgumentParser()
    p.add_argument("asm")
    p.add_argument("kernel")
    p.add_argument("--file", default="plumtree.hip")
    p.add_argument("--loop", default=None)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    lines = open(a.asm).read().splitlines()
    files = {}
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', ln) or re.match(r'\s*\.file\s+(\d+)\s+"([^"]+)"', ln)
        if m:
            files[m.group(1)] = m.group(2)
    start = next(i for i, ln in enumerate(lines) if ln.startswith(a.kernel + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end + 1]
    if a.loop:
        # the loop's blocks: its header and every block whose label comment names
        # it (";   in Loop: Header=BB.. " / "Parent Loop BB.."), nested loops included
        name = a.loop.lstrip(".L")
        keep, inside = [], False
        for i, ln in enumerate(body):
            if re.match(r"^\.?L?BB\d+_\d+:|^; %bb\.\d+:", ln):
                inside = ln.startswith(a.loop + ":") or ("Header=" + name + " ") in ln or ln.rstrip().endswith(
                    "Header=" + name) or ("Loop " + name + " ") in ln or ln.rstrip().endswith("Loop " + name)
                # a numbered block continues the one before it (fallthrough) unless it names another loop
                if ln.startswith("; %bb.") and "in Loop" not in ln:
                    inside = keep[-1] if keep else False
            keep.append(inside)
        body = [ln for ln, k in zip(body, keep) if k]
    cur = None
    cnt = collections.defaultdict(lambda: collections.Counter())
    for ln in body:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            f = files.get(m.group(1), m.group(1))
            cur = (f.split("/")[-1], int(m.group(2)))
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cls = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") and not op.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop")) else
               "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "scratch_", "flat_")) else "other")
        cnt[cur][cls] += 1
        cnt[cur]["all"] += 1
    tot = collections.Counter()
    for c in cnt.values():
        tot.update(c)
    print("total", dict(tot))
    rows = sorted(cnt.items(), key=lambda kv: -(kv[1]["VALU"] + kv[1]["SALU"]))
    src = {}
    for (f, l), c in rows[: a.top]:
        if f and f.endswith(a.file) and f not in src:
            try:
                src[f] = open(f).read().splitlines()
            except OSError:
                src[f] = []
        text = src.get(f, [])
        code = text[l - 1].strip()[:70] if f in src and 0 < l <= len(text) else ""
        print(f"{str(f)[-14:]:>14}:{l:<5} VALU {c['VALU']:4d} SALU {c['SALU']:4d} other {c['all'] - c['VALU'] - c['SALU']:4d}  {code}")


if __name__ == "__main__":
    main()
