"""Multi-process runs of the C ABI under the ftrun launcher (test infrastructure).

`run_probe` writes per-rank inputs, launches `ftrun -np P ftar_probe` against either the
host-sim build (CPU tests of the host logic) or the product libftar.so (GPU parity), and
collects per-rank outputs and statuses for comparison with the oracle.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import tempfile
from dataclasses import dataclass

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTSIM = os.path.join(ROOT, "tests", "hostsim", "_build")
# the same host-sim build with AddressSanitizer + UndefinedBehaviorSanitizer (test_sanitizers.py)
HOSTSIM_ASAN = os.path.join(ROOT, "tests", "hostsim", "_build_asan")
PKG = os.path.join(ROOT, "fault-tolerant_amd")


@dataclass
class ProbeRun:
    returncode: int
    stdout: str
    stderr: str
    outputs: dict      # rank -> list of np arrays (one per iteration)
    status: dict       # rank -> list of (rc, comm_rank, comm_size, recoveries, wall_us)

    @property
    def aborted(self) -> bool:
        return "MPI_ABORT" in self.stderr


def reap_shm(prefix: str = "ftarhs-") -> int:
    """Remove host-sim segments (/dev/shm/ftarhs-<tag>-<pid>-<seq>) whose owner process is
    gone -- what a killed or timed-out job leaves behind; segments of live processes (another
    pytest-xdist worker's job) stay.  Returns the number removed."""
    n = 0
    for f in glob.glob(f"/dev/shm/{prefix}*"):
        parts = os.path.basename(f).rsplit("-", 2)
        if len(parts) != 3 or not parts[1].isdigit():
            continue
        try:
            os.kill(int(parts[1]), 0)
            continue  # the owner lives
        except ProcessLookupError:
            pass
        except PermissionError:
            continue
        try:
            os.unlink(f)
            n += 1
        except OSError:
            pass
    return n


def kill_env(kills) -> str:
    """(rank, phase, step, point[, call]) tuples -> FTAR_KILL."""
    return ",".join(":".join(str(v) for v in k) for k in kills)


# The options a test pins when it asserts a FORM (mesh_steps, gate counts, one-shot use) rather
# than only the result: the suite runs under any FTAR_MESH / FTAR_PUSH / FTAR_TREE_UNROLL / FTAR_GATE
# setting of its environment -- e.g. the node's chosen transport made the default -- and only the
# tests that say which form they check pin it.
MESH_FORM = {"FTAR_MESH": "1", "FTAR_PUSH": "0", "FTAR_TREE_UNROLL": "1", "FTAR_MESH_WAIT": "1"}
# FTAR_GPU_WIDE=1: the GPU suite's repeats of a shape already covered once (more forms, seeds,
# sizes) -- off by default so the suite stays well inside the driver's time limit (VERDICT r04
# next #5); every BASELINE config still runs at full size once without it.
WIDE = os.environ.get("FTAR_GPU_WIDE") == "1"


def wide(*cases):
    """Parametrize values that run only under FTAR_GPU_WIDE=1."""
    return list(cases) if WIDE else []
GATES_ON = {"FTAR_GATE": "1", "FTAR_FLAG_SYNC": "1"}


def run_probe(algo: str, inputs, kills=(), op: int = 0, iters: int = 1, backend: str = "hostsim",
              timeout: int = 120, devmap: str | None = None, env_extra: dict | None = None) -> ProbeRun:
    p = len(inputs)
    dt = {np.dtype(np.int32): 0, np.dtype(np.float32): 1, np.dtype(np.int64): 2,
          np.dtype(np.float64): 3}[inputs[0].dtype]
    count = inputs[0].size
    tmp = tempfile.mkdtemp(prefix="ftar_probe_")
    try:
        for r, x in enumerate(inputs):
            np.ascontiguousarray(x).tofile(os.path.join(tmp, f"in_{r}.bin"))
        if backend in ("hostsim", "hostsim_asan"):
            hs = HOSTSIM if backend == "hostsim" else HOSTSIM_ASAN
            ftrun = os.path.join(hs, "bin", "ftrun")
            probe = os.path.join(hs, "bin", "ftar_probe")
        else:  # "gpu": the product library; "gpu_hooks": its TEST-ONLY hooks build (FTAR_KILL_WITHDRAW)
            ftrun = os.path.join(PKG, "bin", "ftrun")
            probe = os.path.join(HOSTSIM, "gpu_hooks" if backend == "gpu_hooks" else "gpu", "ftar_probe")
        env = dict(os.environ)
        tag = os.path.basename(tmp)
        env.update(FTAR_PROBE_DIR=tmp, FTAR_PROBE_ALGO=algo, FTAR_PROBE_DTYPE=str(dt),
                   FTAR_PROBE_OP=str(op), FTAR_PROBE_COUNT=str(count), FTAR_PROBE_ITERS=str(iters),
                   FTAR_HOSTSIM_TAG=tag)
        env.pop("FTAR_KILL", None)
        if kills:
            env["FTAR_KILL"] = kill_env(kills)
        if env_extra:
            env.update(env_extra)
        cmd = [ftrun, "-np", str(p)]
        if devmap:
            cmd += ["--devmap", devmap]
        cmd += [probe]
        cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
        outs, stats = {}, {}
        for r in range(p):
            for it in range(iters):
                f = os.path.join(tmp, f"out_{r}_{it}.bin")
                s = os.path.join(tmp, f"status_{r}_{it}.txt")
                if os.path.exists(f) and os.path.exists(s):
                    outs.setdefault(r, []).append(np.fromfile(f, dtype=inputs[0].dtype))
                    stats.setdefault(r, []).append(tuple(int(v) for v in open(s).read().split()))
        return ProbeRun(cp.returncode, cp.stdout, cp.stderr, outs, stats)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
        for f in glob.glob(f"/dev/shm/ftarhs-{os.path.basename(tmp)}-*"):
            try:
                os.unlink(f)
            except OSError:
                pass


def run_driver(which: str, nprocs: int, count: int, backend: str = "hostsim", kills=(),
               env_extra: dict | None = None, timeout: int = 120):
    """Run the drop-in src/<which>/main under ftrun and parse its stdout."""
    if backend == "hostsim":
        ftrun = os.path.join(HOSTSIM, "bin", "ftrun")
        exe = os.path.join(HOSTSIM, "src", which, "main")
    else:
        ftrun = os.path.join(PKG, "bin", "ftrun")
        exe = os.path.join(PKG, "src", which, "main")
    env = dict(os.environ)
    env["FTAR_HOSTSIM_TAG"] = f"drv{os.getpid()}"
    env.pop("FTAR_KILL", None)
    if kills:
        env["FTAR_KILL"] = kill_env(kills)
    if env_extra:
        env.update(env_extra)
    try:
        cp = subprocess.run([ftrun, "-np", str(nprocs), exe, str(count)], env=env, capture_output=True,
                            text=True, timeout=timeout)
    finally:  # also on TimeoutExpired: every rank's fake device memory
        for f in glob.glob(f"/dev/shm/ftarhs-drv{os.getpid()}-*"):
            try:
                os.unlink(f)
            except OSError:
                pass
    hello = {}
    for line in cp.stdout.splitlines():
        t = line.split()
        if t and t[0] == "Hello":
            hello[int(t[2])] = int(t[-1])
    return cp, hello


def run_torch_worker(algo: str, inputs, devmap: str, env_extra: dict | None = None, timeout: int = 300) -> ProbeRun:
    """Run tests/device_worker.py (torch tensors on the GPU, the device-pointer entry
    points) as `len(inputs)` ranks under the product's ftrun; two calls per rank."""
    import sys
    p = len(inputs)
    tmp = tempfile.mkdtemp(prefix="ftar_torch_")
    try:
        for r, x in enumerate(inputs):
            np.ascontiguousarray(x, dtype=np.float32).tofile(os.path.join(tmp, f"in_{r}.bin"))
        env = dict(os.environ, FTAR_PROBE_DIR=tmp, FTAR_PROBE_ALGO=algo)
        env.pop("FTAR_KILL", None)
        if env_extra:
            env.update(env_extra)
        cmd = [os.path.join(PKG, "bin", "ftrun"), "-np", str(p), "--devmap", devmap, sys.executable, "-u",
               os.path.join(ROOT, "tests", "device_worker.py")]
        cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
        outs, stats = {}, {}
        for r in range(p):
            for it in range(2):
                f = os.path.join(tmp, f"out_{r}_{it}.bin")
                s = os.path.join(tmp, f"status_{r}_{it}.txt")
                if os.path.exists(f) and os.path.exists(s):
                    outs.setdefault(r, []).append(np.fromfile(f, dtype=np.float32))
                    stats.setdefault(r, []).append(tuple(int(v) for v in open(s).read().split()))
        return ProbeRun(cp.returncode, cp.stdout, cp.stderr, outs, stats)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def with_specials(ins, seed):
    """NaN, signed zeros and infinities at random places: MAX/MIN results then depend on
    the operand order of every combination, so bit equality pins the reduction tree."""
    rng = np.random.default_rng(seed)
    sp = np.array([np.nan, -0.0, 0.0, np.inf, -np.inf], dtype=ins[0].dtype)
    out = []
    for x in ins:
        x = x.copy()
        idx = rng.choice(x.size, size=x.size // 8, replace=False)
        x[idx] = rng.choice(sp, size=idx.size)
        out.append(x)
    return out
