"""C3 cost split by phase and message kind: runs the C3 probe
(tools/probe_engines.py c3: 1M peers, SCAMP v2 c = 5, 5 % crash/rejoin churn
per round, a heartbeat every 10 rounds) on the diagnostic build
partisan_amd/exp_c3prof.so (make -C partisan_amd/csrc c3prof: -DC3_PROF, the
kernels clock their phases per wave with s_memtime and count the messages
they handle by kind), and prints the churn rounds' split.

Cycles are per-wave phase durations summed over waves (a wave's phase ends
when its last lane leaves it), so the shares say where the waves spend their
time; SIMD concurrency makes the sum exceed the kernel's wall time.

usage: python tools/c3_prof.py [n] [churn_rounds]   (GPU box)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SC_KIND = {1: "forward_subscription", 2: "keep_subscription", 3: "ping", 4: "remove_subscription",
           5: "replace_subscription", 6: "bootstrap_remove"}
PD_KIND = {1: "broadcast", 2: "prune", 3: "i_have", 4: "ignored_i_have", 5: "graft"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    env = dict(os.environ, PSIM_LIB_PATH=os.path.join(ROOT, "partisan_amd", "exp_c3prof.so"))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_engines.py"), "c3", str(n)], env=env,
                       capture_output=True, text=True, check=True)
    line = json.loads(p.stdout.strip().splitlines()[-1])
    sc = [list(map(int, ln.split()[1:])) for ln in p.stderr.splitlines() if ln.startswith("sc_prof")]
    pd = [list(map(int, ln.split()[1:])) for ln in p.stderr.splitlines() if ln.startswith("pd_prof")]
    # the churn rounds are the last `rounds` rounds of each engine
    d = lambda x: [a - b for a, b in zip(x[-1], x[-1 - rounds])]  # noqa: E731
    s, t = d(sc), d(pd)
    sc_tot = sum(s[0:4])
    pd_tot = sum(t[0:5])
    out = {
        "config": "C3", "n": n, "churn_rounds": rounds, "build": "exp_c3prof.so (-DC3_PROF)",
        "probe": line,
        "sc_process": {
            "phase_share": {k: round(s[i] / sc_tot, 3) for i, k in enumerate(("calls (joins/leaves)", "inbox sort",
                                                                               "inbox handlers", "periodic (pings)"))},
            "messages_by_kind_per_round": {SC_KIND[k]: s[4 + k] / rounds for k in SC_KIND},
            "draws_per_round": {"calls": s[11] / rounds, "inbox": s[12] / rounds, "periodic": s[13] / rounds},
            "vertices_with_calls_per_round": s[15] / rounds,
            "wave_cycles_per_round": sc_tot / rounds,
        },
        "pd_process": {
            "phase_share": {k: round(t[i] / pd_tot, 3) for i, k in enumerate(("load + updates", "inbox sort",
                                                                               "inbox handlers", "lazy tick (rows)",
                                                                               "compact + store"))},
            "load_share": round(t[13] / pd_tot, 3),
            "messages_by_kind_per_round": {PD_KIND[k]: t[5 + k] / rounds for k in PD_KIND},
            "rows_walked_per_round": t[11] / rounds,
            "update_events_per_round": t[14] / rounds,
            "wave_cycles_per_round": pd_tot / rounds,
        },
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
