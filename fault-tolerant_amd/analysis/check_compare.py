"""Compare-campaign checker: the counterpart of the reference's analysis/check_compare.py.

Reads the stdout of one (NP, SIZE) point of the campaign -- the fault-tolerant drivers
(../out/rd.txt, ../out/raben.txt) and the vendor baselines (../out/original_rd.txt,
../out/original_raben.txt) -- and, when every rank of both runs printed the same
checksum, appends `NP;SIZE;TIME;RESULT` to ../data/data_compare/{rd,original_rd,raben,
original_raben}.csv (the reference's layout, analysis/check_compare.py:4-12,44-51);
otherwise it records both runs in ../out/error.txt.

Stdout grammar (rd/recursive_doubling.c:146-149): `P: <N>`, `Size: <count>`,
`Time: <s>`, `Hello from <r> of <N> and the result is: <checksum>`.  The last P/Size/
Time line wins; every Hello line contributes one result.

Directories can be moved with FTAR_CMP_OUT (default ../out) and FTAR_CMP_DATA
(default ../data/data_compare).
"""
from __future__ import annotations

import csv
import os

OUT = os.environ.get("FTAR_CMP_OUT", "../out")
DATA = os.environ.get("FTAR_CMP_DATA", "../data/data_compare")
PAIRS = (("rd", "original_rd", "RD"), ("raben", "original_raben", "RABEN"))
HEADER = ["NP", "SIZE", "TIME", "RESULT"]


def parse(path: str):
    """-> (np, size, time, [results]); missing fields stay None."""
    np_, size, t, results = None, None, None, []
    try:
        text = open(path).read()
    except OSError:
        return np_, size, t, results
    for line in text.splitlines():
        tok = line.split()
        if not tok:
            continue
        try:
            if tok[0] == "Hello":
                results.append(int(tok[-1]))
            elif tok[0] == "P:":
                np_ = int(tok[-1])
            elif tok[0] == "Size:":
                size = int(tok[-1])
            elif tok[0] == "Time:":
                t = float(tok[-1])
        except ValueError:
            continue
    return np_, size, t, results


def consistent(a: list, b: list, np_) -> bool:
    """Both runs have one result per rank and every result equals the first one."""
    if np_ is None or len(a) != np_ or len(b) != np_:
        return False
    return all(v == a[0] for v in a) and all(v == a[0] for v in b)


def append_row(path: str, row):
    new = not os.path.exists(path)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "a", newline="") as f:
        w = csv.writer(f, delimiter=";")
        if new:
            w.writerow(HEADER)
        w.writerow(row)


def check_pair(ft: str, orig: str, label: str) -> bool:
    a = parse(os.path.join(OUT, f"{ft}.txt"))
    b = parse(os.path.join(OUT, f"{orig}.txt"))
    if consistent(a[3], b[3], a[0]):
        append_row(os.path.join(DATA, f"{ft}.csv"), [a[0], a[1], a[2], a[3][0]])
        append_row(os.path.join(DATA, f"{orig}.csv"), [b[0], b[1], b[2], b[3][0]])
        print(f"{label}: {a[2]}, {label}_ORG: {b[2]}")
        return True
    with open(os.path.join(OUT, "error.txt"), "a") as f:
        f.write(f"{label}: {[a[0], a[1], a[2], a[3]]}\n")
        f.write(f"{label}_O: {[b[0], b[1], b[2], b[3]]}\n")
        f.write("#" * 45 + "\n")
    print(f"########### ERROR WITH {label} ###########")
    return False


def main() -> int:
    np_, size, _, res = parse(os.path.join(OUT, "rd.txt"))
    print(f"NP: {np_}, SIZE: {size}, RESULT: {res[0] if res else None}")
    ok = [check_pair(*p) for p in PAIRS]
    print("#" * 52)
    return 0 if all(ok) else 1


if __name__ == "__main__":
    raise SystemExit(main())
