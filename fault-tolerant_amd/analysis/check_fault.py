"""Classify one fault-injection run and append it to a CSV log.

Drop-in for the reference's analysis/check_fault.py: same invocation
(`python3 ../analysis/check_fault.py <rd|raben> <log.csv>` from run/), same inputs
(../out/test_log.txt, ../out/mpi_out.txt, ../out/docker_out.txt), same outputs
(../out/check.txt, ../out/log_errors.txt on a deadlock or wrong result, and one
`;`-separated row N;DELAY;BUF SIZE;KILLED;TIME;DEADLOCK;SEGFAULT;ABORT;RIGHT RESULT).

Rules restated from the reference:
  expected checksum  ((N(N-1)/2) % 17) * BUF_SIZE -- the dead ranks' inputs included
  DEADLOCK           bash `time` real > TIMEOUT
  ABORT              a line starting with MPI_ABORT, or an MPI_ERRORS_ARE_FATAL token
  SEGFAULT           "Segmentation fault" or "(core dumped)" in the test log
  KILLED             N - number of distinct ranks that printed "Hello"
  TIME               the last "Time:" printed by a rank, else the `time` real value
Beside the row, <log.csv>.victims gets N;KILLED;VICTIMS;MID EXCHANGE from the launcher's
post mortem (ftrun prints, for every rank killed by a signal, whether a kernel reading
peers' HBM was in flight): the GPU exchange takes milliseconds, so whether a random kill
met data movement is recorded rather than assumed.
"""
import csv
import os
import re
import sys

OUT = os.path.join("..", "out")
HEADER = ["N", "DELAY", "BUF SIZE", "KILLED", "TIME", "DEADLOCK", "SEGFAULT", "ABORT", "RIGHT RESULT"]


def expected_checksum(n_ranks, buf_size):
    value = ((n_ranks * (n_ranks - 1) / 2) % 17) * buf_size
    print(value, int(value))
    return int(value)


def parse_real(token):
    """bash `time` prints e.g. 0m3.214s."""
    m = re.match(r"(?:(\d+)m)?([\d.]+)s", token)
    if not m:
        return None
    return 60.0 * float(m.group(1) or 0) + float(m.group(2))


def read_test_log(path):
    info = {"segfault": False, "abort": False, "real": None, "victims": []}
    with open(path) as f:
        for raw in f:
            m = re.match(r"ftrun: rank (\d+) \(pid \d+\) killed by signal \d+ (.*)", raw.strip())
            if m:  # the launcher's post mortem of a killed rank (not in the reference)
                info["victims"].append((int(m.group(1)), m.group(2).startswith("mid-exchange")))
            if "Segmentation fault" in raw or "(core dumped)" in raw:
                info["segfault"] = True
            tok = raw.split()
            if not tok:
                continue
            key = tok[0]
            if key in ("N", "BUF_SIZE", "DELAY", "TIMEOUT") and len(tok) >= 3:
                info[key] = float(tok[-1]) if key == "DELAY" else int(tok[-1])
            elif key == "real":
                info["real"] = parse_real(tok[-1])
            elif key == "MPI_ABORT" or "MPI_ERRORS_ARE_FATAL" in tok:
                info["abort"] = True
    return info


def read_job_output(path, n_ranks, expected):
    survivors, right, last_time = set(), True, None
    with open(path) as f:
        for raw in f:
            tok = raw.split()
            if not tok:
                continue
            if tok[0] == "Hello":
                survivors.add(int(tok[2]))
                if int(tok[-1]) != expected:
                    right = False
            elif tok[0] == "Time:":
                last_time = float(tok[-1])
    killed = sum(1 for r in range(n_ranks) if r not in survivors)
    return killed, right, last_time


def keep_logs(algo, row, target=os.path.join(OUT, "log_errors.txt")):
    with open(target, "a") as out:
        out.write(f"Algo Used: {algo}\n")
        for name in ("mpi_out.txt", "docker_out.txt", "test_log.txt"):
            p = os.path.join(OUT, name)
            if os.path.exists(p):
                out.write(open(p).read() + "\n")
        out.write("\n" + str(row))
        out.write("\n" + "#" * 70)


def main(argv):
    algo, log_file = argv[1], argv[2]
    info = read_test_log(os.path.join(OUT, "test_log.txt"))
    n, buf = info["N"], info["BUF_SIZE"]
    expected = expected_checksum(n, buf)
    killed, right, t = read_job_output(os.path.join(OUT, "mpi_out.txt"), n, expected)
    real = info["real"] if info["real"] is not None else 0.0
    deadlock = real > info.get("TIMEOUT", 30)
    row = [n, info["DELAY"], buf, killed, t if t is not None else real, deadlock, info["segfault"], info["abort"],
           right]
    with open(os.path.join(OUT, "check.txt"), "w") as f:
        f.write("True" if (killed == 1 and right and not deadlock) else "False")
    print(row)
    if deadlock or not right:
        keep_logs(algo, row)
        print("########################### ERROR ###########################")
    new = not os.path.exists(log_file)
    with open(log_file, "a", newline="") as f:
        w = csv.writer(f, delimiter=";")
        if new:
            w.writerow(HEADER)
        w.writerow(row)
    # Row-side log (the reference's CSV grammar stays untouched): which ranks the launcher
    # saw killed by a signal and whether each died mid-exchange, one line per CSV row.
    side = log_file + ".victims"
    new = not os.path.exists(side)
    with open(side, "a", newline="") as f:
        w = csv.writer(f, delimiter=";")
        if new:
            w.writerow(["N", "KILLED", "VICTIMS", "MID EXCHANGE"])
        v = info["victims"]
        w.writerow([n, killed, " ".join(str(r) for r, _ in v), any(mid for _, mid in v) if v else ""])


if __name__ == "__main__":
    main(sys.argv)
