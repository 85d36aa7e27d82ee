"""Tables of the two campaigns -- the counterpart of the reference's analysis/
analyze_compare.py, analyze_fault.py and clean_data.py, on the CSVs this build writes
(check_compare.py / check_fault.py).

    python analyze.py compare <ft.csv> <original.csv> [--label L] [--plot out.png]
        mean TIME per (NP, SIZE) of both, and the FT / original ratio
        (analyze_compare.py:19-39)
    python analyze.py fault <log.csv> [--max-time 5]
        count / mean / median / std / max of TIME per (N, KILLED), rows with TIME below
        the cut only (analyze_fault.py:6-14,30-35)
    python analyze.py clean <in.csv> <out.csv> N [N ...]
        at most 50 rows per (N, KILLED in {0, 1}), random.Random-seeded 42 sample
        (clean_data.py:4-35)

Plots are written only with --plot and only if matplotlib is importable (it is not
part of this image); the tables are the product.
"""
from __future__ import annotations

import argparse
import csv
import random
import sys

import pandas as pd


def compare_table(ft_csv: str, orig_csv: str, label: str = "FT") -> pd.DataFrame:
    a = pd.read_csv(ft_csv, sep=";").groupby(["NP", "SIZE"], as_index=False)["TIME"].mean()
    b = pd.read_csv(orig_csv, sep=";").groupby(["NP", "SIZE"], as_index=False)["TIME"].mean()
    m = pd.merge(a, b, on=["NP", "SIZE"], suffixes=(f"_{label}", "_ORIGINAL"))
    m[f"RATIO_{label}"] = m[f"TIME_{label}"] / m["TIME_ORIGINAL"]
    return m.sort_values(["NP", "SIZE"]).reset_index(drop=True)


def fault_table(log_csv: str, max_time: float = 5.0) -> pd.DataFrame:
    df = pd.read_csv(log_csv, delimiter=";")
    for c in ("N", "KILLED", "TIME"):
        df[c] = pd.to_numeric(df[c], errors="coerce")
    df = df.dropna(subset=["N", "KILLED", "TIME"])
    df = df[df["TIME"] < max_time]
    g = df.groupby(["N", "KILLED"])["TIME"].agg(["count", "mean", "median", "std", "max"])
    return g.reset_index()


def clean(in_csv: str, out_csv: str, ns, per_class: int = 50) -> int:
    with open(in_csv, newline="", encoding="utf-8") as f:
        data = list(csv.DictReader(f, delimiter=";"))
    out = []
    for n in ns:
        rows = [r for r in data if int(r["N"]) == n]
        k0 = [r for r in rows if int(r["KILLED"]) == 0]
        k1 = [r for r in rows if int(r["KILLED"]) == 1]
        random.seed(42)
        out += random.sample(k0, min(per_class, len(k0)))
        out += random.sample(k1, min(per_class, len(k1)))
    with open(out_csv, "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=list(data[0].keys()) if data else [], delimiter=";")
        w.writeheader()
        w.writerows(out)
    return len(out)


def _plot_compare(m: pd.DataFrame, label: str, path: str) -> bool:
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print("matplotlib not available: no plot", file=sys.stderr)
        return False
    nps = sorted(m["NP"].unique())
    fig, axes = plt.subplots(nrows=1, ncols=len(nps) + 1, figsize=(5 * (len(nps) + 1), 4))
    for ax, n in zip(axes, nps):
        s = m[m["NP"] == n]
        ax.loglog(s["SIZE"] * 4, s[f"TIME_{label}"], marker="o", label=label)
        ax.loglog(s["SIZE"] * 4, s["TIME_ORIGINAL"], marker="s", label="vendor")
        ax.set_title(f"NP = {n}")
        ax.set_xlabel("bytes")
        ax.legend()
    for n in nps:
        s = m[m["NP"] == n]
        axes[-1].semilogx(s["SIZE"] * 4, s[f"RATIO_{label}"], marker="o", label=f"NP={n}")
    axes[-1].set_title("FT / vendor time")
    axes[-1].legend()
    fig.tight_layout()
    fig.savefig(path)
    return True


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("compare")
    c.add_argument("ft_csv")
    c.add_argument("orig_csv")
    c.add_argument("--label", default="FT")
    c.add_argument("--plot", default=None)
    f = sub.add_parser("fault")
    f.add_argument("log_csv")
    f.add_argument("--max-time", type=float, default=5.0)
    k = sub.add_parser("clean")
    k.add_argument("in_csv")
    k.add_argument("out_csv")
    k.add_argument("ns", type=int, nargs="+")
    a = ap.parse_args(argv)
    if a.cmd == "compare":
        m = compare_table(a.ft_csv, a.orig_csv, a.label)
        print(m.to_string(index=False))
        if a.plot:
            _plot_compare(m, a.label, a.plot)
    elif a.cmd == "fault":
        print(fault_table(a.log_csv, a.max_time).to_string(index=False, float_format="{:.3f}".format))
    else:
        print(f"kept {clean(a.in_csv, a.out_csv, a.ns)} rows -> {a.out_csv}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
