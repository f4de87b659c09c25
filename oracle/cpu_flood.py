"""CPU baseline worker for bench.py (TEST/MEASUREMENT INFRASTRUCTURE ONLY:
the oracle is timed here as the reported CPU baseline, never shipped).

One process = one single-threaded C oracle (oracle/plumtree.c) flooding a
random overlay to quiescence; bench.py runs W of them at once (spawned
interpreters) to report the host's all-core throughput beside the
single-thread figure (SURVEY 8(d) "CPU baseline timing")."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def flood(job):
    n, peers, seed, reps, lazy = job
    import pyoracle as O
    from partisan_amd import overlay
    rp, col = overlay.random_regular(n, peers, seed)
    pr, secs, rounds = 0, 0.0, 0
    for _ in range(reps):
        orc = O.Plumtree(rp, col, lazy)
        t0 = time.perf_counter()
        orc.heartbeat(0)
        _, rounds = orc.run()
        secs += time.perf_counter() - t0
        pr += n * rounds
        orc.close()
    return pr, secs, rounds


if __name__ == "__main__":
    # bench.py runs each worker as a plain child process (no multiprocessing
    # pool: its resource tracker outlived the bench) and reads
    # the one JSON line it prints
    import json
    print(json.dumps(flood(tuple(int(x) for x in sys.argv[1:6]))), flush=True)
