"""Random multi-failure sweep on the host-sim: the product vs the oracle, bit for bit.

Draws sets of kill points ((rank, phase, step, point), distinct ranks) at random, keeps
those the oracle recovers from with the requested number of deaths, and runs each through
the host-sim build of the library (real processes, the product's host C).  MAX/MIN over
NaN / signed zeros / infinities pin the operand order of every combination, so a
recovery that takes a different path than the oracle shows up even when the values agree.
This sweep found the new-entry state hand-off and the BARRIER co-victim wait (DESIGN.md
§3, "Second failure after a promotion").

usage: python tests/fault_sweep.py [--p 11] [--kills 2] [--draws 400] [--seed 3] [--jobs 6] [--aborts]
                                  [--spread 8] [--withdraw]
--spread K puts rank r on device r % K (the node's layout: the auto redundancy moves Raben's
step-0 copy), --withdraw has each victim retract its input as it dies (a lost device's memory).
"""
import argparse
import os
import random
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import harness as H  # noqa: E402
import oracle as O  # noqa: E402


def run_one(algo, p, op, kills, count, aborts=False, devmap=None, env=None):
    ins = H.with_specials(O.random_inputs(p, count, seed=p + 78), p + 4)
    fn = O.rabenseifner if algo == "raben" else O.recursive_doubling
    o = fn(ins, list(kills), op=op)
    if o.aborted and not aborts:
        return None
    if not o.aborted and sum(s == O.DEAD for s in o.status) < len(kills):
        return None
    try:
        r = H.run_probe(algo, ins, list(kills), op=op, backend="hostsim", timeout=30, devmap=devmap, env_extra=env)
    except Exception:
        return "hang"
    if o.aborted:  # the product must abort too (MPI_Abort line, no survivor output)
        return "ok" if r.aborted and not r.outputs else "did not abort"
    if r.aborted:
        return "aborted"
    bad = [w for w in range(p) if o.status[w] == 0 and
           (w not in r.outputs or not np.array_equal(r.outputs[w][0].view(np.uint32), o.outputs[w].view(np.uint32)))]
    return bad or "ok"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=11)
    ap.add_argument("--kills", type=int, default=2)
    ap.add_argument("--draws", type=int, default=400)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--count", type=int, default=1031)
    ap.add_argument("--jobs", type=int, default=6)
    ap.add_argument("--aborts", action="store_true", help="also run the draws the oracle aborts (must abort)")
    ap.add_argument("--spread", type=int, default=0, help="rank r on device r %% K (0: every rank on device 0)")
    ap.add_argument("--withdraw", action="store_true", help="victims retract their input as they die")
    a = ap.parse_args()
    rnd = random.Random(a.seed)
    nst = max(3, a.p.bit_length() - 1)  # every step of the schedule (L = floor(log2 p)), at least 3
    pts = [(v, ph, st, pt) for v in range(a.p) for ph in (1, 2) for st in range(nst) for pt in range(4)]
    cases = []
    for algo in ("raben", "rd"):
        for _ in range(a.draws):
            ks = tuple(rnd.sample(pts, a.kills))
            if len({k[0] for k in ks}) == a.kills:
                cases.append((algo, a.p, rnd.choice([0, 2, 3]), ks, a.count))
    with ThreadPoolExecutor(a.jobs) as ex:
        devmap = ",".join(str(r % a.spread) for r in range(a.p)) if a.spread > 0 else None
        env = {"FTAR_KILL_WITHDRAW": "1"} if a.withdraw else None
        res = list(ex.map(lambda c: run_one(*c, aborts=a.aborts, devmap=devmap, env=env), cases))
    ran = [(c, r) for c, r in zip(cases, res) if r is not None]
    bad = [(c, r) for c, r in ran if r != "ok"]
    what = "recovering or aborting" if a.aborts else "recovering"
    print(f"{len(cases)} drawn, {len(ran)} {what} with {a.kills} deaths, {len(bad)} differ from the oracle")
    for c, r in bad[:20]:
        print("  ", c[0], "op", c[2], "kills", c[3], "->", r)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
