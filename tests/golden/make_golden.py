"""Extract small golden fixtures from the reference's recorded results (data files only).

Sources (read as CSV text; no reference code is imported or run):
  /root/reference/data/data_compare/{rd,raben,original_rd,original_raben}.csv
      NP;SIZE;TIME;RESULT -- RESULT is the per-rank checksum sum_i(result[i] % 17) printed by
      src/{rd,raben}/main (int32 SUM, buffer[i] = rank), identical on every rank.
  /root/reference/data/data_fault/log_single_{RD,Raben}.csv
      N;DELAY;BUF SIZE;KILLED;TIME;DEADLOCK;SEGFAULT;ABORT;RIGHT RESULT -- outcomes of the
      random single-kill campaign (run/run_test.sh with kill=1).

Outputs (committed):
  ref_checksums.csv       algo;NP;SIZE;RESULT  (one row per combination, every recorded SIZE up to
                          the campaign's maximum 2^27)
  ref_fault_outcomes.csv  algo;N;KILLED;ABORT;DEADLOCK;RIGHT;count
"""
import collections
import csv
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rows = {}
    for algo in ("rd", "raben", "original_rd", "original_raben"):
        with open(os.path.join(REF, "data_compare", f"{algo}.csv")) as f:
            for r in csv.DictReader(f, delimiter=";"):
                np_, size, res = int(r["NP"]), int(r["SIZE"]), int(r["RESULT"])
                rows.setdefault((algo, np_, size), res)
    with open(os.path.join(HERE, "ref_checksums.csv"), "w") as f:
        f.write("algo;NP;SIZE;RESULT\n")
        for (algo, np_, size), res in sorted(rows.items()):
            f.write(f"{algo};{np_};{size};{res}\n")
    cnt = collections.Counter()
    for algo, fn in (("rd", "log_single_RD.csv"), ("raben", "log_single_Raben.csv")):
        with open(os.path.join(REF, "data_fault", fn)) as f:
            for r in csv.DictReader(f, delimiter=";"):
                cnt[(algo, int(r["N"]), int(r["KILLED"]), r["ABORT"], r["DEADLOCK"], r["RIGHT RESULT"])] += 1
    with open(os.path.join(HERE, "ref_fault_outcomes.csv"), "w") as f:
        f.write("algo;N;KILLED;ABORT;DEADLOCK;RIGHT;count\n")
        for k, v in sorted(cnt.items()):
            f.write(";".join(str(x) for x in k) + f";{v}\n")


if __name__ == "__main__":
    main()
