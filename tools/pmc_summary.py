"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_summary.json.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes), with the gfx950
correction of MI355X_MICROARCH.md section HBM: FETCH_SIZE counts exactly half of the bytes
of a wide (16 B/lane) coalesced streaming read; WRITE_SIZE is exact for 16-B stores.
Each counter comes from its own rocprofv3 pass (they do not fit one pass together).

usage: python tools/pmc_summary.py <name> <kernel-substring> <fetch_csv> <write_csv> [out.json]

Each entry records where it was measured (`measured_at`: the CSVs, the git HEAD of the tree
and the date), which bench.py reports as the roofline's `traffic_source`.
"""
import csv
import json
import os
import subprocess
import sys
import time


def mean_counter(path, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def head():
    try:
        return subprocess.run(["git", "-C", os.path.dirname(os.path.abspath(__file__)), "rev-parse", "--short", "HEAD"],
                              capture_output=True, text=True, timeout=10).stdout.strip() or None
    except (OSError, subprocess.SubprocessError):
        return None  # the GPU box's copy of the tree has no .git


def main():
    name, kernel, fcsv, wcsv = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                               "pmc_summary.json")
    fetch, nf = mean_counter(fcsv, "FETCH_SIZE", kernel)
    write, nw = mean_counter(wcsv, "WRITE_SIZE", kernel)
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[name] = {"kernel": kernel, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "launches": [nf, nw],
               "hbm_bytes_per_launch": round((2 * fetch + write) * 1024) if fetch and write else None,
               "correction": "2*FETCH_SIZE (gfx950 half-count on 16B/lane streams) + WRITE_SIZE, KiB->B",
               "measured_at": {"fetch_csv": fcsv, "write_csv": wcsv, "head": head(), "date": time.strftime("%Y-%m-%d")}}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d[name]))


if __name__ == "__main__":
    main()
