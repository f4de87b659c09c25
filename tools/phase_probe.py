"""Phases of the ELL round kernel's workgroup 0, launch by launch, for one
10M-peer flood (diagnostic): needs the PSIM_PHASE_PROF variant library
(make -C partisan_amd/csrc variant NAME=phase DEFS=-DPSIM_PHASE_PROF=1; run
with PSIM_LIB_PATH=tools/ab/libpsim_phase.so).

Columns (us, 100 MHz real-time ticks): counts = entry -> round counts read,
list = -> first chunk's groups known, sweep = -> its words in LDS, cand = ->
its candidates listed, loop = -> its candidate loop done, rest = -> all
chunks done, flush = -> counters flushed; period = this launch's entry - the
previous launch's entry.

usage: PSIM_LIB_PATH=... python tools/phase_probe.py [--n 10000000] [--steps 3]"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import partisan_amd as pa  # noqa: E402
from partisan_amd._lib import lib  # noqa: E402


def phases():
    L = lib()
    f = L.psim_debug_phases
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_uint32, C.POINTER(C.c_uint32)]
    cap = 4096
    buf = (C.c_ulonglong * (cap * 8))()
    n = C.c_uint32(0)
    if f(buf, cap, C.byref(n)) != 0:
        raise SystemExit("psim_debug_phases failed")
    return [list(buf[8 * i:8 * i + 8]) for i in range(n.value)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--peers", type=int, default=5)
    p.add_argument("--steps", type=int, default=3)
    a = p.parse_args()
    rp, col = pa.overlay.random_regular(a.n, a.peers, 0x5EED0001)
    sim = pa.Simulator()
    sim.load_overlay(rp, col)
    sim.set_chunk_timing(False)                   # an event pair per round kernel
    for step in range(a.steps):
        sim.reset_trees()
        sim.broadcast(0)
        phases()                                  # drop earlier launches
        st, r = sim.run()
    recs = phases()
    print(f"n={a.n} rounds={r} launches recorded={len(recs)}")
    names = ["counts", "list", "sweep", "cand", "loop", "rest", "flush"]
    print(f"{'L':>3} {'kern_us':>8} " + " ".join(f"{x:>7}" for x in names) + f" {'period':>8} {'msgs':>9}")
    prev = None
    for i, t in enumerate(recs):
        row = []
        last = t[0]
        for j in range(1, 8):
            if t[j]:
                row.append(f"{(t[j] - last) / 100.0:7.2f}")
                last = t[j]
            else:
                row.append(f"{'-':>7}")
        per = f"{(t[0] - prev) / 100.0:8.2f}" if prev else f"{'-':>8}"
        prev = t[0]
        ms = st[i]["kernel_ms"] * 1e3 if i < len(st) else 0.0
        m = sum(st[i][k] for k in pa._lib.MSG_KINDS.values()) if i < len(st) else 0
        print(f"{i + 1:>3} {ms:8.2f} " + " ".join(row) + f" {per} {m:9d}")
    sim.close()


if __name__ == "__main__":
    main()
