"""The drop-in harness (run/run_test.sh -> run_mpi.sh -> ftrun + killer -> check_fault.py)
end to end on CPU, with the host-sim rank executables.  The killer is swapped for
tests/scoped_kill.sh (same policy, restricted to this job's processes)."""
import csv
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fault-tolerant_amd")


def _run_test(tmp_path, kill, algo, n_range=(5, 9)):
    log = tmp_path / f"{algo}_{kill}.csv"
    env = dict(os.environ, FTAR_NMIN=str(n_range[0]), FTAR_NMAX=str(n_range[1]), FTAR_BUF_MAX="200000",
               FTAR_LOOP_SECONDS="3.5", FTAR_KILLER=os.path.join(ROOT, "tests", "scoped_kill.sh"),
               USER=os.environ.get("USER", "root"), FTAR_HOSTSIM_TAG="harness")
    exe = os.path.relpath(os.path.join(ROOT, "tests", "hostsim", "_build", "src", algo, "main"),
                          os.path.join(PKG, "run"))
    cp = subprocess.run(["./run_test.sh", str(kill), str(log), algo, exe], cwd=os.path.join(PKG, "run"), env=env,
                        capture_output=True, text=True, timeout=120)
    subprocess.run("rm -f /dev/shm/ftarhs-harness-*", shell=True)
    rows = list(csv.DictReader(open(log), delimiter=";"))
    return cp, rows


@pytest.fixture(autouse=True)
def _clean_out():
    yield
    shutil.rmtree(os.path.join(PKG, "out"), ignore_errors=True)
    shutil.rmtree(os.path.join(PKG, "log"), ignore_errors=True)


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_no_kill_right_result(hostsim, tmp_path, algo):
    cp, rows = _run_test(tmp_path, 0, algo)
    assert len(rows) == 1, cp.stdout + cp.stderr
    r = rows[0]
    assert r["KILLED"] == "0" and r["RIGHT RESULT"] == "True" and r["DEADLOCK"] == "False", r
    assert r["ABORT"] == "False" and r["SEGFAULT"] == "False"


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_single_kill_is_classified(hostsim, tmp_path, algo):
    """One random rank killed mid-run: the row is either a recovery (KILLED=1, right
    result including the dead rank's data) or a clean MPI_Abort (KILLED=N) -- the two
    outcome classes of the reference's campaign; never a deadlock or a wrong result."""
    cp, rows = _run_test(tmp_path, 1, algo)
    r = rows[0]
    n = int(r["N"])
    assert r["DEADLOCK"] == "False" and r["SEGFAULT"] == "False", cp.stdout + cp.stderr
    assert r["RIGHT RESULT"] == "True"
    assert (r["KILLED"] == "1" and r["ABORT"] == "False") or (r["ABORT"] == "True" and int(r["KILLED"]) == n) \
        or r["KILLED"] == "0", r


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_multiple_kill_is_classified(hostsim, tmp_path, algo):
    """KILL=2 (run_mpi.sh picks 1..N-1 victims, killed 0.5 s apart): a recovery with the
    right result, or a clean MPI_Abort -- never a deadlock, a crash or a wrong result."""
    cp, rows = _run_test(tmp_path, 2, algo)
    assert len(rows) == 1, cp.stdout + cp.stderr
    r = rows[0]
    assert r["DEADLOCK"] == "False" and r["SEGFAULT"] == "False", (r, cp.stdout + cp.stderr)
    assert r["RIGHT RESULT"] == "True", r
