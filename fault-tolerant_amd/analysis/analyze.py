"""Tables and figures of the two campaigns -- the counterpart of the reference's
analysis/analyze_compare.py, analyze_fault.py, analyze_log.py and clean_data.py, on the
CSVs this build writes (check_compare.py / check_fault.py) and on bench.py's JSON line.

    python analyze.py compare <ft.csv> <original.csv> [--label L] [--plot out.png]
        mean TIME per (NP, SIZE) of both and the FT / original ratio; the figure is one
        time-vs-size panel per NP plus the ratio panel (analyze_compare.py:18-99)
    python analyze.py fault <log.csv> [--max-time 5] [--label L] [--plot out.png]
        count / mean / median / std / max of TIME per (N, KILLED), rows with TIME below
        the cut; the figure is the 0-vs-1-killed boxplot per N (analyze_fault.py:6-71)
    python analyze.py outcomes <log.csv> [--plot out.png]
        outcome classes of the runs with a kill -- recovered, recovered-then-abort,
        abort, wrong result, deadlock -- as a table and a pie (analyze_log.py)
    python analyze.py sweep <bench.json> [--plot out.png]
        bench.py's N > 1 size sweep (4 B .. 256 MiB): FT Rabenseifner / recursive
        doubling per-call time and, on the 8-GPU node, RCCL's all_reduce and the FT/RCCL
        ratio -- the compare campaign's curve measured inside the driver's run
    python analyze.py clean <in.csv> <out.csv> N [N ...]
        at most 50 rows per (N, KILLED in {0, 1}), random.Random-seeded 42 sample
        (clean_data.py:4-35)

Figures use matplotlib's Agg backend (file output, no display).
"""
from __future__ import annotations

import argparse
import csv
import json
import random

import pandas as pd


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def human_bytes(b: float) -> str:
    b = int(b)
    for unit, k in (("GiB", 1 << 30), ("MiB", 1 << 20), ("KiB", 1 << 10)):
        if b >= k:
            return f"{b // k}{unit}"
    return f"{b}B"


def compare_table(ft_csv: str, orig_csv: str, label: str = "FT") -> pd.DataFrame:
    a = pd.read_csv(ft_csv, sep=";").groupby(["NP", "SIZE"], as_index=False)["TIME"].mean()
    b = pd.read_csv(orig_csv, sep=";").groupby(["NP", "SIZE"], as_index=False)["TIME"].mean()
    m = pd.merge(a, b, on=["NP", "SIZE"], suffixes=(f"_{label}", "_ORIGINAL"))
    m[f"RATIO_{label}"] = m[f"TIME_{label}"] / m["TIME_ORIGINAL"]
    return m.sort_values(["NP", "SIZE"]).reset_index(drop=True)


def fault_frame(log_csv: str, max_time: float = 5.0) -> pd.DataFrame:
    df = pd.read_csv(log_csv, delimiter=";")
    for c in ("N", "KILLED", "TIME"):
        df[c] = pd.to_numeric(df[c], errors="coerce")
    df = df.dropna(subset=["N", "KILLED", "TIME"])
    return df[df["TIME"] < max_time]


def fault_table(log_csv: str, max_time: float = 5.0) -> pd.DataFrame:
    g = fault_frame(log_csv, max_time).groupby(["N", "KILLED"])["TIME"].agg(["count", "mean", "median", "std", "max"])
    return g.reset_index()


def outcome_counts(log_csv: str) -> dict:
    """Runs with at least one kill, classified like analyze_log.py: deadlock, wrong
    result, abort with survivors (a rank recovered, then the job aborted), abort of the
    whole job, recovered."""
    c = {"recovered": 0, "abort_after_recovery": 0, "abort": 0, "wrong_result": 0, "deadlock": 0}
    with open(log_csv, newline="") as f:
        for r in csv.DictReader(f, delimiter=";"):
            if r["KILLED"] == "0":
                continue
            survived = int(r["N"]) - int(r["KILLED"])
            if r["DEADLOCK"] == "True":
                c["deadlock"] += 1
            elif r["RIGHT RESULT"] == "False":
                c["wrong_result"] += 1
            elif r["ABORT"] == "True":
                c["abort_after_recovery" if survived > 0 else "abort"] += 1
            else:
                c["recovered"] += 1
    return c


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


def plot_compare(m: pd.DataFrame, label: str, path: str, ticks: int = 8) -> None:
    plt = _plt()
    nps = sorted(m["NP"].unique())
    ncols = 2
    nrows = (len(nps) + ncols) // ncols
    fig, axes = plt.subplots(nrows=nrows, ncols=ncols, figsize=(12, 4 * nrows), squeeze=False)
    axes = axes.flatten()
    sizes = sorted(m["SIZE"].unique())
    idx = sorted({int(round(i * (len(sizes) - 1) / max(1, ticks - 1))) for i in range(ticks)})
    tick_sizes = [sizes[i] * 4 for i in idx]
    for ax, n in zip(axes, nps):
        s = m[m["NP"] == n].sort_values("SIZE")
        ax.plot(s["SIZE"] * 4, s[f"TIME_{label}"], marker="o", label=label)
        ax.plot(s["SIZE"] * 4, s["TIME_ORIGINAL"], marker="s", label=f"vendor ({label})")
        ax.set_xscale("log")
        ax.set_yscale("log")
        ax.set_title(f"NP = {n}")
        ax.set_xlabel("message size")
        ax.set_ylabel("mean time (s)")
        ax.set_xticks(tick_sizes)
        ax.set_xticklabels([human_bytes(t) for t in tick_sizes], rotation=45, ha="right")
        ax.grid(True)
        ax.legend()
    r = axes[-1]
    for n in nps:
        s = m[m["NP"] == n].sort_values("SIZE")
        r.plot(s["SIZE"] * 4, s[f"RATIO_{label}"], marker="o", label=f"NP={n}")
    r.set_xscale("log")
    r.set_xticks(tick_sizes)
    r.set_xticklabels([human_bytes(t) for t in tick_sizes], rotation=45, ha="right")
    r.set_title("FT / vendor time")
    r.set_ylabel("time ratio")
    r.grid(True, linestyle="--", alpha=0.7)
    r.legend()
    for j in range(len(nps), len(axes) - 1):
        fig.delaxes(axes[j])
    fig.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)


def plot_fault(df: pd.DataFrame, label: str, path: str) -> None:
    import matplotlib.patches as mpatches
    plt = _plt()
    ns = sorted(df["N"].unique())
    pos = list(range(len(ns)))
    w = 0.35
    fig = plt.figure(figsize=(max(6, 1.6 * len(ns) + 3), 5))
    mean = dict(marker="D", markeredgecolor="black", markerfacecolor="black", markersize=6)
    for k, (shift, color) in enumerate(((-w / 2, "#1f77b4"), (w / 2, "#ff7f0e"))):
        data = [df[(df["N"] == n) & (df["KILLED"] == k)]["TIME"].values for n in ns]
        keep = [i for i, d in enumerate(data) if len(d)]
        if keep:
            plt.boxplot([data[i] for i in keep], positions=[pos[i] + shift for i in keep], widths=w,
                        patch_artist=True, showmeans=True, meanprops=mean,
                        boxprops=dict(facecolor=color, alpha=0.8), medianprops=dict(color="black"))
    plt.xticks(pos, [str(int(n)) for n in ns])
    plt.xlabel("number of ranks (N)")
    plt.ylabel("time (s)")
    plt.yscale("log")
    plt.title(f"{label}: zero vs one killed rank")
    plt.legend(handles=[mpatches.Patch(color="#1f77b4", alpha=0.8, label="without failures"),
                        mpatches.Patch(color="#ff7f0e", alpha=0.8, label="one rank killed")], loc="upper left")
    plt.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)


def plot_outcomes(c: dict, path: str, title: str = "single-kill outcomes") -> None:
    plt = _plt()
    items = [(k, v) for k, v in c.items() if v]
    fig = plt.figure(figsize=(6, 5))
    plt.pie([v for _, v in items], labels=[f"{k} ({v})" for k, v in items], autopct="%1.1f%%")
    plt.title(title)
    fig.savefig(path, dpi=110)
    plt.close(fig)


def sweep_table(bench_json: str) -> pd.DataFrame:
    with open(bench_json) as f:
        d = json.loads([l for l in f.read().splitlines() if l.startswith("{")][-1])
    rows = [v for v in d.get("size_sweep_us", {}).values() if isinstance(v, dict)]  # (skip the setting keys)
    t = pd.DataFrame(rows).sort_values("bytes").reset_index(drop=True)
    t.attrs["n_gpus"] = d.get("n_gpus")
    return t


def plot_sweep(t: pd.DataFrame, path: str) -> None:
    plt = _plt()
    fig, axes = plt.subplots(1, 2, figsize=(12, 4.5))
    ax = axes[0]
    for col, lab, mk in (("raben_us", "FT Rabenseifner", "o"), ("rd_us", "FT recursive doubling", "^"),
                         ("raben_no_oneshot_us", "FT Rabenseifner, two-launch mesh", "."),
                         ("rccl_us", "RCCL all_reduce", "s")):
        if col in t and t[col].notna().any():
            ax.plot(t["bytes"], t[col], marker=mk, label=lab)
    ax.set_xscale("log", base=2)
    ax.set_yscale("log")
    ax.set_xlabel("bytes per rank")
    ax.set_ylabel("time per call (us), max over ranks")
    ax.set_title(f"per-call time, {t.attrs.get('n_gpus')} ranks")
    ax.grid(True)
    ax.legend()
    ax = axes[1]
    if "raben_over_rccl" in t and t["raben_over_rccl"].notna().any():
        ax.plot(t["bytes"], t["raben_over_rccl"], marker="o", label="FT Rabenseifner / RCCL")
        ax.set_ylabel("time ratio")
        ax.set_title("FT / vendor (the compare campaign's ratio)")
    else:
        ax.plot(t["bytes"], t["bytes"] / t["raben_us"] / 1e3, marker="o", label="FT Rabenseifner")
        ax.set_ylabel("algbw (GB/s)")
        ax.set_title("algorithmic bandwidth (no RCCL column in this run)")
    ax.set_xscale("log", base=2)
    ax.grid(True)
    ax.legend()
    fig.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)


def _last_line(path: str) -> dict:
    with open(path) as f:
        return json.loads([l for l in f.read().splitlines() if l.startswith("{")][-1])


def decisions(line: dict) -> dict:
    """What one N > 1 bench line (the driver's node run) decides for the next build
    (DESIGN.md 9.1): the mesh form its transport selection picked, whether the mid-size
    gates pay (the largest size up to which every gated column beats its ungated twin:
    FTAR_OPT_GATE_MAX), whether configs[4]'s elided step-0 copy recovered across GPUs
    (deviation 6), which small-call setting was exact, and the north-star fractions."""
    sel = line.get("transport_selection") or {}
    sweep = {int(k): v for k, v in (line.get("size_sweep_us") or {}).items() if isinstance(v, dict)}
    gate_max = 1 << 20  # the library's default
    for b in sorted(k for k in sweep if k > (1 << 20)):
        row = sweep[b]
        pairs = [(row.get(f"{a}_midgate_us"), row.get(f"{a}_us")) for a in ("raben", "rd")]
        pairs = [(g, u) for g, u in pairs if g is not None and u is not None]
        if not pairs or any(g >= u for g, u in pairs):
            break
        gate_max = b
    ns = line.get("north_star") or {}
    c5 = line.get("c5_single_kill") or {}
    ex = line.get("exact_on_node") or {}
    times = {k[:-3]: v for k, v in sel.items() if k.endswith("_ms")}
    rdl = (line.get("rd") or {}).get("schedule_link_roofline") or {}
    return {
        "n_gpus": line.get("n_gpus"),
        "rehearsal": bool(ns.get("rehearsal")),
        "value_GBps": line.get("value"),
        "transport_chosen": sel.get("chosen", line.get("transport")),
        "transport_ms": times,
        "transport_inexact_or_failed": sorted(set(sel.get("inexact") or []) | set(sel.get("failed") or {})),
        "never_fastest": sorted(k for k in times if k != sel.get("chosen")),
        # the allgather ordered on the device (the default) vs after a host agree (FTAR_OPT_MESH_WAIT=0)
        "device_wait_faster": (times["mesh"] < times["mesh_host_ag"]) if "mesh_host_ag" in times and "mesh" in times
        else None,
        "gate_max_bytes": gate_max,
        "gate_max_changes": gate_max != (1 << 20),
        "all_exact": ex.get("all_exact"),
        "small_call_setting": (line.get("size_sweep_us") or {}).get("small_call_setting"),
        "dead_input_cross_device": c5.get("dead_input_cross_device"),
        "elide_step0_copy_across_gpus": c5.get("dead_input_cross_device") == "recovered",
        "north_star_frac": ns.get("frac"),
        "north_star_met": ns.get("met"),
        "reference_schedule_frac": ns.get("reference_schedule_frac"),
        "north_star_non_kernel_ms": ns.get("non_kernel_ms"),
        "north_star_frac_kernels_only": ns.get("frac_kernels_only"),
        "rd_transport": rdl.get("transport"),
        "rd_frac": rdl.get("frac"),
        "rd_reference_schedule_frac": rdl.get("reference_schedule_frac"),
        "link_GBps": (line.get("link_calibration") or {}).get("single_link_GBps"),
    }


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
    f.add_argument("--label", default="FT Allreduce")
    f.add_argument("--plot", default=None)
    o = sub.add_parser("outcomes")
    o.add_argument("log_csv")
    o.add_argument("--plot", default=None)
    s = sub.add_parser("sweep")
    s.add_argument("bench_json")
    s.add_argument("--plot", default=None)
    d = sub.add_parser("decisions", help="what the node's N > 1 bench lines decide (DESIGN.md 9.1)")
    d.add_argument("bench_json", nargs="+")
    k = sub.add_parser("clean")
    k.add_argument("in_csv")
    k.add_argument("out_csv")
    k.add_argument("ns", type=int, nargs="+")
    a = ap.parse_args(argv)
    if a.cmd == "compare":
        m = compare_table(a.ft_csv, a.orig_csv, a.label)
        print(m.to_string(index=False))
        if a.plot:
            plot_compare(m, a.label, a.plot)
    elif a.cmd == "fault":
        print(fault_table(a.log_csv, a.max_time).to_string(index=False, float_format="{:.3f}".format))
        if a.plot:
            plot_fault(fault_frame(a.log_csv, a.max_time), a.label, a.plot)
    elif a.cmd == "outcomes":
        cnt = outcome_counts(a.log_csv)
        print(json.dumps(cnt))
        if a.plot:
            plot_outcomes(cnt, a.plot)
    elif a.cmd == "sweep":
        t = sweep_table(a.bench_json)
        print(t.to_string(index=False))
        if a.plot:
            plot_sweep(t, a.plot)
    elif a.cmd == "decisions":
        for path in a.bench_json:
            print(json.dumps(decisions(_last_line(path))))
    else:
        print(f"kept {clean(a.in_csv, a.out_csv, a.ns)} rows -> {a.out_csv}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
