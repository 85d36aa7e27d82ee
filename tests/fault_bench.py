"""C5 on one GPU box: Raben Allreduce with a single injected kill, recovery cost.

Runs 9 ranks (8 + one idle spare, SURVEY.md 8d layout) of the probe under ftrun, all on
GPU 0 (the 8-GPU node is not available to this script), three calls per job:
call 0 warm-up, call 1 carries the kill (when given), call 2 runs on the survivors.
Reports per-call wall time of rank 0 for the no-fault job and the fault job, and checks
every survivor's result against the oracle.

usage: python tests/fault_bench.py [count] [victim phase step point]
FTAR_FB_RANKS=p changes the rank count (default 9).  More than 8 rank processes on the
one GPU exceed its hardware contexts and get time-sliced (calls of 0.1-30 s); p = 5
(4 + one idle spare) keeps the C5 structure within them.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import harness as H  # noqa: E402
import oracle as O  # noqa: E402


NRANKS = int(os.environ.get("FTAR_FB_RANKS", "9"))


def run(count, kill):
    ins = O.random_inputs(NRANKS, count, seed=5)
    kills = [kill + (1,)] if kill else []
    r = H.run_probe("raben", ins, kills, iters=3, backend="gpu", devmap=",".join(["0"] * NRANKS), timeout=600)
    o = O.rabenseifner(ins, [kill] if kill else [])
    ok = not r.aborted
    for w in range(NRANKS):
        if o.status[w] == 0 and ok:
            ok &= np.array_equal(r.outputs[w][1].view(np.uint32), o.outputs[w].view(np.uint32))
    walls = [st[4] / 1e3 for st in r.status.get(0, [])]
    per_rank = {w: [{"wall_ms": s[4] / 1e3, "sync_ms": s[5] / 1e3, "drain_ms": s[6] / 1e3, "syncs": s[7]}
                    for s in r.status[w]] for w in r.status}
    return {"kill": kill, "aborted": r.aborted, "parity_ok": bool(ok), "rank0_call_ms": walls,
            "recoveries": [st[3] for st in r.status.get(0, [])], "per_rank": per_rank}


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 24)
    kill = tuple(int(v) for v in sys.argv[2:6]) if len(sys.argv) > 5 else (5, 1, 1, 0)
    res = {"ranks": NRANKS, "count": count, "bytes": count * 4, "nofault": run(count, None), "fault": run(count, kill)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
