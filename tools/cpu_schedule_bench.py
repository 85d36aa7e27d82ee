"""CPU baseline of the schedules: the build's own C host logic -- control
plane, agree rounds, both FT schedules -- run as N host processes, one pinned per core,
with POSIX shared memory as the transport and plain C loops as the reduce
(tests/hostsim: the product's C sources linked against the host-memory device layer,
built with -O3 -march=x86-64-v3).  Reported beside the GPU numbers, never as them.

    python tools/cpu_schedule_bench.py [--quick] [--out FILE]

Configs: C1 (p = 4, 64 KiB int32, both schedules, the reference's driver case) and
256 MiB float32 at p = 2 / 4 / 8 when the host has that many cores.  Time = the
drivers' `Time:` line (wall clock of one call incl. copy-in/out), max over ranks,
median over repetitions.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import resource
import signal
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HS = os.path.join(ROOT, "tests", "hostsim")
OUT = "_build_o3"


def build():
    # x86-64-v3 (AVX2), not -march=native: the binaries are built here and run on the GPU
    # box's host CPU, a different microarchitecture
    subprocess.run(["make", "-s", "-C", HS, f"OUT={OUT}", "CFLAGS=-O3 -march=x86-64-v3 -g -std=c11 -Wall "
                    "-Wno-unused-parameter -fPIC -D_GNU_SOURCE", f"{OUT}/src/rd/main", f"{OUT}/src/raben/main",
                    f"{OUT}/bin/ftrun"], check=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run_proc(cmd, env, timeout):
    """The job in a process group of its own, SIGKILLed as a whole past `timeout`."""
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
        return p.returncode, out, err, False
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        return p.returncode, out, err, True


def run(algo: str, p: int, count: int, dtype: str, reps: int, timeout: float = 1800.0) -> dict:
    """`reps` calls of the schedule, all of them within `timeout` seconds (a job still
    running then is killed with its ranks and the run fails)."""
    deadline = time.monotonic() + timeout
    exe = os.path.join(HS, OUT, "src", algo, "main")
    ftrun = os.path.join(HS, OUT, "bin", "ftrun")
    # the reference's shape: pairwise exchanges step by step (no relay, no mesh)
    env = dict(os.environ, FTAR_PIN_CPUS="1", FTAR_HOSTSIM_TAG=f"cpub{os.getpid()}", FTAR_DTYPE=dtype,
               FTAR_MESH="0", FTAR_RELAY="0")
    times, cpu = [], []
    for _ in range(reps):
        ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        rc, out, err, timed_out = run_proc([ftrun, "-np", str(p), exe, str(count)], env,
                                           max(1.0, deadline - time.monotonic()))
        subprocess.run(f"rm -f /dev/shm/ftarhs-cpub{os.getpid()}-*", shell=True)
        if timed_out:
            raise TimeoutError(f"{algo} p={p}: still running after {timeout:.0f} s (killed)")
        if rc != 0:
            raise RuntimeError(f"{algo} p={p} failed: {err[-1000:]}")
        ts = [float(x) for x in re.findall(r"^Time: (\S+)", out, flags=re.M)]
        hello = re.findall(r"result is: (-?\d+)", out)
        expect = ((p * (p - 1) // 2) % 17) * count
        if len(hello) != p or any(int(h) != expect for h in hello):
            raise RuntimeError(f"{algo} p={p}: wrong checksums {hello} (expected {expect})")
        times.append(max(ts))
        ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        cpu.append((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / p)
    t = statistics.median(times)
    S = count * 4
    return {"algo": algo, "p": p, "count": count, "dtype": dtype, "reps": reps, "time_s": t,
            "algbw_GBps": round(S / t / 1e9, 4), "times_s": times,
            # the reference's TIME is clock() of one rank; ranks here spin, so CPU time per
            # rank tracks wall time (this figure also covers init, fill and checksum)
            "cpu_s_per_rank_whole_process": round(statistics.median(cpu), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="C1 only (seconds)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    build()
    ncpu = len(os.sched_getaffinity(0))
    res = {"kind": "port (product host C + host-memory device layer, one process per core, pairwise step-by-step "
                   "exchanges as in the reference)",
           "cpu_model": cpu_model(), "cpus": ncpu, "results": []}
    t0 = time.time()
    for algo in ("rd", "raben"):
        res["results"].append(run(algo, 4, 16384, "int32", 20))
    if not args.quick:
        for p in (2, 4, 8):
            if p > ncpu:
                continue
            for algo in ("rd", "raben"):
                res["results"].append(run(algo, p, 67108864, "float32", 3))
                print(json.dumps(res["results"][-1]), file=sys.stderr, flush=True)
    res["wall_s"] = round(time.time() - t0, 1)
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
