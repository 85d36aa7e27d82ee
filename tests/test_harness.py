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
    # the row-side log: the launcher's post mortem names the victim and whether it died
    # with a pull in flight (the padded steps re-pull their windows, so it mostly does)
    side = list(csv.DictReader(open(str(tmp_path / f"{algo}_1.csv") + ".victims"), delimiter=";"))
    assert len(side) == 1 and side[0]["N"] == r["N"] and side[0]["KILLED"] == r["KILLED"], side
    if r["KILLED"] == "1":
        assert len(side[0]["VICTIMS"].split()) == 1 and side[0]["MID EXCHANGE"] in ("True", "False"), side


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_multiple_kill_is_classified(hostsim, tmp_path, algo):
    """KILL=2 (run_mpi.sh picks 1..N-1 victims, killed 0.5 s apart): a recovery with the
    right result, or a clean MPI_Abort -- never a deadlock, a crash or a wrong result."""
    cp, rows = _run_test(tmp_path, 2, algo)
    assert len(rows) == 1, cp.stdout + cp.stderr
    r = rows[0]
    assert r["DEADLOCK"] == "False" and r["SEGFAULT"] == "False", (r, cp.stdout + cp.stderr)
    assert r["RIGHT RESULT"] == "True", r


def test_launcher_never_a_kill_candidate(hostsim):
    """run_mpi.sh passes the rank program through FTAR_PROG, so the reference killer's
    rule (run/kill_procs.sh:12: R-state processes whose command line contains "main")
    matches the rank processes but never `timeout` or the ftrun launcher, which sleeps in
    sigtimedwait.  Sampled over a 2 s stretched run of a 4-rank job."""
    import time
    exe = os.path.join(ROOT, "tests", "hostsim", "_build", "src", "raben", "main")
    env = dict(os.environ, FTAR_PROG=exe, FTAR_LOOP_SECONDS="2", FTAR_HOSTSIM_TAG=f"kc{os.getpid()}")
    proc = subprocess.Popen(["timeout", "30", os.path.join(ROOT, "tests", "hostsim", "_build", "bin", "ftrun"),
                             "-np", "4", "50000"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    seen_ranks, launchers, bad = set(), set(), set()
    try:
        t0 = time.time()
        while proc.poll() is None and time.time() - t0 < 20:
            rows = []
            for line in subprocess.run(["ps", "-e", "-o", "pid=,ppid=,stat=,args="], capture_output=True,
                                       text=True).stdout.splitlines():
                f = line.split(None, 3)
                if len(f) == 4:
                    rows.append((int(f[0]), int(f[1]), f[2], f[3]))
            tree = {proc.pid}
            changed = True
            while changed:
                changed = False
                for pid, ppid, _, _ in rows:
                    if ppid in tree and pid not in tree:
                        tree.add(pid)
                        changed = True
            for pid, ppid, st, args in rows:
                if pid not in tree:
                    continue
                if ppid == proc.pid:
                    launchers.add(pid)
                if "main" in args and st.startswith("R"):  # the reference killer's candidates
                    (bad if pid == proc.pid or ppid == proc.pid else seen_ranks).add(pid)
            time.sleep(0.02)
        out, err = proc.communicate(timeout=30)
    finally:
        if proc.poll() is None:
            proc.kill()
        subprocess.run(f"rm -f /dev/shm/ftarhs-kc{os.getpid()}-*", shell=True)
    assert proc.returncode == 0, err[-2000:]
    assert launchers, "launcher never observed"
    assert not bad, (bad, launchers)
    assert seen_ranks, "no rank process was ever a candidate"
    assert out.count("Hello from") == 4


def test_random_kills_land_mid_exchange(hostsim, tmp_path):
    """The stretched steps (FTAR_LOOP_SECONDS) re-pull their last peer window instead of
    idling, so the reference killer's SIGKILL (a random R-state rank after DELAY) meets a
    pull in flight: at least half of the kills are reported mid-exchange by the launcher."""
    import re
    import time
    exe = os.path.join(ROOT, "tests", "hostsim", "_build", "src", "raben", "main")
    ftrun = os.path.join(ROOT, "tests", "hostsim", "_build", "bin", "ftrun")
    mid = total = 0
    for k in range(6):
        env = dict(os.environ, FTAR_PROG=exe, FTAR_LOOP_SECONDS="2", FTAR_HOSTSIM_TAG=f"mx{os.getpid()}")
        proc = subprocess.Popen([ftrun, "-np", "5", "2000000"], env=env, stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE, text=True)
        try:
            time.sleep(0.8 + 0.15 * k)
            kids = subprocess.run(["ps", "-o", "pid=", "--ppid", str(proc.pid)], capture_output=True,
                                  text=True).stdout.split()
            if kids:
                os.kill(int(kids[k % len(kids)]), 9)
            out, err = proc.communicate(timeout=60)
        finally:
            if proc.poll() is None:
                proc.kill()
            subprocess.run(f"rm -f /dev/shm/ftarhs-mx{os.getpid()}-*", shell=True)
        post = re.findall(r"ftrun: rank \d+ \(pid \d+\) killed by signal 9 (.*)", err)
        total += len(post)
        mid += sum(1 for p in post if p.startswith("mid-exchange"))
    assert total >= 4, total
    assert mid * 2 >= total, (mid, total)


def test_compare_outcomes_classes(tmp_path):
    """tools/compare_outcomes.py: a campaign's check_fault.py rows classified as the
    reference's fixture rows are (recovered / abort / no death / deadlock / wrong result) and
    tabled beside them per (schedule, N)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("compare_outcomes", os.path.join(ROOT, "tools", "compare_outcomes.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    d = tmp_path / "camp" / "n12"
    d.mkdir(parents=True)
    hdr = "N;DELAY;BUF SIZE;KILLED;TIME;DEADLOCK;SEGFAULT;ABORT;RIGHT RESULT\n"
    (d / "log_single_RD.csv").write_text(hdr + "12;2.0;100;1;4.0;False;False;False;True\n"
                                         "12;3.0;100;12;4.0;False;False;True;True\n"
                                         "12;3.0;100;12;30.0;True;False;False;True\n")
    (d / "log_nokill_RD.csv").write_text(hdr + "12;2.0;100;0;4.0;False;False;False;True\n"
                                         "12;2.0;100;0;4.0;False;False;False;False\n")
    out = tmp_path / "o.md"
    m.main(["x", str(out), str(tmp_path / "camp")])
    text = out.read_text()
    assert "### rd N = 12" in text
    rows = {l.split("|")[1].strip(): l for l in text.splitlines() if l.startswith("| ")}
    for cls, n in (("recovered", 1), ("abort", 1), ("deadlock", 1), ("no death", 1), ("wrong result", 1)):
        assert rows[cls].split("|")[2].strip().startswith(f"{n} ("), (cls, rows[cls])
    # the reference's RD N = 12 rows (tests/golden/ref_fault_outcomes.csv): 50 recovered, 250 aborts
    assert rows["recovered"].split("|")[3].strip().startswith("50 (")
    assert rows["abort"].split("|")[3].strip().startswith("250 (")
