"""Outcome classes of a fault campaign (check_fault.py rows) beside the reference's own.

    python tools/compare_outcomes.py OUT.md CAMPAIGN_DIR...

Reads every log_{single,nokill}_{RD,Raben}.csv under the campaign directories and
tests/golden/ref_fault_outcomes.csv (the reference's data/data_fault rows, classified the same
way), and writes one markdown table per (schedule, N): recovered with the right result
(KILLED = 1), clean abort (ABORT, every rank gone), deadlock, wrong result, no death (KILLED =
0), counts and shares.  Classes are comparable, counts are not: the reference drew its kill
delays against seconds-long CPU exchanges, this harness against a stretched GPU schedule
(run/run_mpi.sh), so the step a kill lands in -- which decides recover or abort -- is drawn
differently.
"""
import csv
import glob
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(killed, n, abort, deadlock, right):
    if deadlock:
        return "deadlock"
    if not right:
        return "wrong result"
    if abort:
        return "abort"
    if killed == 0:
        return "no death"
    return "recovered" if killed < n else "abort"


def ours(dirs):
    out = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "log_*_*.csv"), recursive=True):
            algo = "rd" if f.endswith("_RD.csv") else "raben"
            for r in csv.DictReader(open(f), delimiter=";"):
                n = int(r["N"])
                c = classify(int(r["KILLED"]), n, r["ABORT"] == "True", r["DEADLOCK"] == "True",
                             r["RIGHT RESULT"] == "True")
                out.setdefault((algo, n), Counter())[c] += 1
    return out


def reference():
    out = {}
    path = os.path.join(ROOT, "tests", "golden", "ref_fault_outcomes.csv")
    for r in csv.DictReader(open(path), delimiter=";"):
        n = int(r["N"])
        c = classify(int(r["KILLED"]), n, r["ABORT"] == "True", r["DEADLOCK"] == "True", r["RIGHT"] == "True")
        out.setdefault((r["algo"], n), Counter())[c] += int(r["count"])
    return out


def table(key, mine, ref):
    classes = ["recovered", "abort", "no death", "deadlock", "wrong result"]
    rows = [f"### {key[0]} N = {key[1]}", "", "| class | this build | reference |", "|---|---|---|"]
    tm, tr = sum(mine.values()), sum(ref.values())
    for c in classes:
        a = f"{mine[c]} ({100 * mine[c] / tm:.0f} %)" if tm else "-"
        b = f"{ref[c]} ({100 * ref[c] / tr:.0f} %)" if tr else "- (no row at this N)"
        rows.append(f"| {c} | {a} | {b} |")
    return rows + [""]


def main(argv):
    out_md, dirs = argv[1], argv[2:]
    mine, ref = ours(dirs), reference()
    lines = ["# Campaign outcome classes beside the reference's", "", __doc__.split("\n\n", 2)[2].strip(), ""]
    for key in sorted(mine):
        lines += table(key, mine[key], ref.get(key, Counter()))
    open(out_md, "w").write("\n".join(lines))
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv)
