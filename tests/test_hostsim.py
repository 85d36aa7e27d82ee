"""CPU tests of the product's host logic, as real multi-process jobs.

The product's host C (control plane, agree/barrier, both schedules, both error
handlers, the ftrun launcher and the drop-in drivers) is linked against a host-memory
device layer (tests/hostsim/dev_host.c, test-only) so every rank is a real process,
failures are real SIGKILLs detected through the robust-mutex failure detector, and the
outcomes are compared with the oracle's simulation of the reference.
"""
import os
import random
import signal
import subprocess
import time

import numpy as np
import pytest

import harness as H
import oracle as O


def _cmp(oracle_fn, algo, inputs, kills=(), op=0, env=None):
    o = oracle_fn(inputs, kills, op=op)
    r = H.run_probe(algo, inputs, kills, op=op, backend="hostsim", timeout=120, env_extra=env)
    u = {4: np.uint32, 8: np.uint64}[inputs[0].dtype.itemsize]
    if all(st == O.DEAD for st in o.status):
        # every rank killed (e.g. p = 1): no survivor to detect it or to call MPI_Abort;
        # the job is lost, as an mpiexec job of killed processes is
        assert not r.outputs and r.returncode != 0, (kills, r.returncode, r.stderr[-1000:])
        return o, r
    if o.aborted:
        assert r.aborted and not r.outputs, (kills, r.stderr[-1000:])
        # the same abort: the handlers' MPI_Abort codes (1 Raben, 16 RD check_abort), 75 where a
        # region under ERRORS_ARE_FATAL sees the failure.  Raben at rem = 0 holds the allgather's
        # last agree and the fatal barrier as one round (ftar_raben.c rb_mesh): a death between
        # them (POST) is seen by the allgather's handler there, which aborts with its own code
        codes = {o.abort_code}
        if algo == "raben" and o.abort_code == 75 and any(k[1] == 3 for k in kills):
            codes.add(1)
        assert any(f"with errorcode {c}." in r.stderr for c in codes), (kills, o.abort_code, r.stderr[-1000:])
        return o, r
    assert not r.aborted, (kills, r.stderr[-1000:])
    for w, st in enumerate(o.status):
        if st == 0:
            assert np.array_equal(r.outputs[w][0].view(u), o.outputs[w].view(u)), (algo, kills, w)
        else:
            assert w not in r.outputs
    return o, r


def _fn(oracle, algo):
    return oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16, 17])
def test_nofault_parity(hostsim, oracle, algo, p):
    _cmp(_fn(oracle, algo), algo, oracle.random_inputs(p, 1031, seed=p))


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("dtype,op", [(np.int32, 0), (np.int64, 1), (np.float64, 2), (np.float32, 3)])
def test_nofault_dtypes_ops(hostsim, oracle, algo, dtype, op):
    _cmp(_fn(oracle, algo), algo, oracle.random_inputs(6, 333, seed=2, dtype=dtype), op=op)


@pytest.mark.parametrize("algo,p", [("raben", 5), ("raben", 9), ("raben", 8), ("rd", 4), ("rd", 6), ("rd", 8),
                                    ("rd", 9)])
def test_single_kill_sweep(hostsim, oracle, algo, p):
    """Every victim x phase x step x point the schedule reaches: same outcome class
    (recover / abort) and bit-identical survivor results."""
    ins = oracle.random_inputs(p, 257, seed=p)
    phases = [0, 1, 2, 3] if algo == "raben" else [0, 1, 3]
    fn = _fn(oracle, algo)
    n = 0
    for v in range(p):
        for ph in phases:
            for st in range(4):
                for pt in range(4):
                    ks = [(v, ph, st, pt)]
                    if fn(ins, ks).status[v] != oracle.DEAD:
                        continue
                    _cmp(fn, algo, ins, ks)
                    n += 1
    assert n > 0


@pytest.mark.parametrize("algo,p", [("raben", 5), ("rd", 6), ("raben", 4)])
def test_host_entry_zero_copy_kill_sweep(hostsim, oracle, algo, p):
    """The _host entry points' zero-copy route (caller buffers pinned: the device entry
    point runs on them in place) under every single kill point: same outcome class and
    bit-identical survivor results as the oracle."""
    ins = oracle.random_inputs(p, 257, seed=p + 40)
    phases = [0, 1, 2, 3] if algo == "raben" else [0, 1, 3]
    fn = _fn(oracle, algo)
    n = 0
    for v in range(p):
        for ph in phases:
            for st in range(3):
                for pt in range(4):
                    ks = [(v, ph, st, pt)]
                    if fn(ins, ks).status[v] != oracle.DEAD:
                        continue
                    _cmp(fn, algo, ins, ks, env={"FTAR_HOSTSIM_PINNED": "1"})
                    n += 1
    assert n > 0


@pytest.mark.parametrize("seed", range(12))
def test_multi_kill_random(hostsim, oracle, seed):
    rng = random.Random(seed)
    algo = rng.choice(["raben", "rd"])
    p = rng.choice([6, 7, 9, 11, 13, 17])
    nk = rng.choice([1, 2, 3])
    victims = rng.sample(range(p), nk)
    kills = [(v, rng.choice([1, 2]) if algo == "raben" else 1, rng.randrange(4), rng.randrange(4)) for v in victims]
    _cmp(_fn(oracle, algo), algo, oracle.random_inputs(p, 511, seed=seed), kills)


def test_repeated_calls_and_retargeted_comm(hostsim, oracle):
    inputs = oracle.random_inputs(5, 2000, seed=2)
    kills = [(3, 1, 1, 2)]
    r = H.run_probe("raben", inputs, kills, iters=3, backend="hostsim")
    o1 = oracle.rabenseifner(inputs, kills)
    assert not r.aborted
    order = o1.order_after
    o2 = oracle.rabenseifner([inputs[w] for w in order])
    for i, w in enumerate(order):
        assert np.array_equal(r.outputs[w][0].view(np.uint32), o1.outputs[w].view(np.uint32))
        assert r.status[w][0][1:4] == (i, 4, 1)      # comm rank, size, recoveries after the call
        for it in (1, 2):
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o2.outputs[i].view(np.uint32))


@pytest.mark.parametrize("p", [4, 8])
def test_rd_repeated_calls_after_recovery(hostsim, oracle, p):
    """RD at a power of two queues every small step's launch ahead of its barrier (gates):
    a recovery in call 0 re-targets the partners, so launches queued for the old plan are
    given up (a gate still closed at the end of the call included); calls 1 and 2 on the
    survivors are exact and gated again where the survivors are a power of two."""
    inputs = oracle.random_inputs(p, 1031, seed=p + 21)
    found = None
    for v in range(p):
        for st in range(p.bit_length() - 1):
            for pt in (0, 2, 3):
                ks = [(v, 1, st, pt)]
                o1 = oracle.recursive_doubling(inputs, ks)
                if not o1.aborted and len(o1.order_after) < p:
                    found = ks, o1
                    break
            if found:
                break
        if found:
            break
    assert found, "no recovering RD kill"
    kills, o1 = found
    # (FTAR_GATE_HOLD_US=0: a loaded test host must not give gates up, the counts are checked)
    r = H.run_probe("rd", inputs, kills, iters=3, backend="hostsim", env_extra={"FTAR_GATE_HOLD_US": "0"})
    assert not r.aborted, r.stderr[-1500:]
    order = o1.order_after
    o2 = oracle.recursive_doubling([inputs[w] for w in order])
    for i, w in enumerate(order):
        assert np.array_equal(r.outputs[w][0].view(np.uint32), o1.outputs[w].view(np.uint32)), w
        assert r.status[w][0][10] >= 1, r.status[w][0]  # call 0 queued step 0 ahead of the kill
        for it in (1, 2):
            st = r.status[w][it]
            assert st[0] == 0, st
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o2.outputs[i].view(np.uint32)), (w, it)
            n = len(order)
            if n & (n - 1) == 0:  # a power of two again: every step gated, none replaced
                assert st[10:12] == (n.bit_length() - 1, 0), st


@pytest.mark.parametrize("algo,p", [("rd", 4), ("raben", 4), ("rd", 8)])
def test_late_peer_gives_the_gate_up(hostsim, oracle, algo, p):
    """A peer that arrives late (here 300 ms) at a call whose small launches are queued
    behind gates: the waiting ranks' barrier passes FTAR_GATE_HOLD_US, so they give their
    gated launch up (the stream is not held by it any longer) and launch after
    the barrier instead -- every result exact, and the give-up counted (gate_holds).  With
    FTAR_GATE_HOLD_US=0 the gate is never given up by the host."""
    ins = oracle.random_inputs(p, 1031, seed=p + 5)
    o = _fn(oracle, algo)(ins)
    late = {"FTAR_PROBE_RANK_ENV": f"{p - 1}:FTAR_PROBE_SLEEP_US=300000", "FTAR_GATE_HOLD_US": "2000"}
    r = H.run_probe(algo, ins, backend="hostsim", iters=3, env_extra=late)
    assert r.returncode == 0, r.stderr[-1000:]
    for w in range(p):
        for it in range(3):
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)
    # (call 0 allocates the workspace: its collective absorbs the late arrival before any gate)
    holds = [r.status[w][it][13] for w in range(p - 1) for it in (1, 2)]
    assert all(h >= 1 for h in holds), r.status
    r = H.run_probe(algo, ins, backend="hostsim", iters=2, env_extra=dict(late, FTAR_GATE_HOLD_US="0"))
    assert r.returncode == 0 and all(r.status[w][it][13] == 0 for w in range(p) for it in range(2)), r.status
    for w in range(p):
        assert np.array_equal(r.outputs[w][1].view(np.uint32), o.outputs[w].view(np.uint32)), w


def test_rd_after_raben_recovery(hostsim, oracle):
    """RD after a Raben recovery runs on the re-targeted comm order."""
    inputs = oracle.random_inputs(9, 777, seed=5)
    kills = [(4, 1, 2, 2)]
    o1 = oracle.rabenseifner(inputs, kills)
    assert not o1.aborted
    r = H.run_probe("raben", inputs, kills, iters=2, backend="hostsim")
    assert not r.aborted
    for w in o1.order_after:
        assert np.array_equal(r.outputs[w][0].view(np.uint32), o1.outputs[w].view(np.uint32))


def test_zero_count_returns_mpi_err_unknown(hostsim, oracle):
    r = H.run_probe("raben", [np.zeros(0, np.float32)] * 3, backend="hostsim")
    assert all(r.status[w][0][0] == 14 for w in range(3))


@pytest.mark.parametrize("which", ["raben", "rd"])
@pytest.mark.parametrize("n", [4, 6, 8, 12, 16])
def test_drivers_match_golden_rows(hostsim, which, n):
    """The drop-in drivers (host-sim device layer) against the reference's recorded
    results: tests/golden/ref_checksums.csv rows for this NP (data/data_compare).  The largest
    size run here keeps the job's vectors within 1 GiB in total (n x size x 4 B): every rank
    holds about 8 vectors of host-sim "device" memory -- its workspace (backed up front, so
    running out is a NOMEM abort, not a rank death), the _host staging and the driver's own
    buffers -- and the container has 64 GiB for the whole suite.  The reference's largest row,
    2^27 ints, runs on the GPU (test_driver_golden_checksums_max_size)."""
    import csv
    with open(os.path.join(H.ROOT, "tests", "golden", "ref_checksums.csv")) as f:
        rows = [r for r in csv.DictReader(f, delimiter=";") if r["algo"] == which and int(r["NP"]) == n]
    sizes = [int(r["SIZE"]) for r in rows]
    assert sizes, "no golden rows"
    big = max(s for s in sizes if n * s * 4 <= (1 << 30))
    for r in rows:
        size = int(r["SIZE"])
        if size not in (1, 3, 64, 16384, 65536, big):
            continue
        cp, hello = H.run_driver(which, n, size)
        assert cp.returncode == 0, cp.stderr
        assert sorted(hello) == list(range(n))
        assert set(hello.values()) == {int(r["RESULT"])}, (size, hello)


@pytest.mark.parametrize("which", ["raben", "rd"])
@pytest.mark.parametrize("n", [4, 5, 6, 8, 9])
def test_drivers_print_reference_lines(hostsim, oracle, which, n):
    cp, hello = H.run_driver(which, n, 16384)
    assert cp.returncode == 0, cp.stderr
    assert sorted(hello) == list(range(n))
    assert set(hello.values()) == {oracle.expected_checksum(n, 16384)}
    lines = cp.stdout.splitlines()
    assert lines.count(f"P: {n}") == n and lines.count("Size: 16384") == n
    assert sum(1 for l in lines if l.startswith("Time: ")) == n
    assert all(l.strip() for l in lines)  # check_fault.py indexes line[0]: no empty lines


def test_driver_float32_mode(hostsim, oracle):
    cp, hello = H.run_driver("raben", 5, 1000, env_extra={"FTAR_DTYPE": "float32"})
    assert set(hello.values()) == {oracle.expected_checksum(5, 1000)}


def test_driver_recovers_and_aborts_like_reference(hostsim, oracle):
    # Raben N=9: a kill in a middle reduce-scatter step is recovered by the idle rank
    cp, hello = H.run_driver("raben", 9, 5000, kills=[(5, 1, 1, 0)])
    assert cp.returncode == 0 and sorted(hello) == [0, 1, 2, 3, 4, 6, 7, 8]
    assert set(hello.values()) == {oracle.expected_checksum(9, 5000)}  # includes the dead rank's data
    # Raben N=8: no idle rank -> MPI_Abort, nobody prints Hello
    cp, hello = H.run_driver("raben", 8, 5000, kills=[(5, 1, 1, 0)])
    assert cp.returncode != 0 and not hello
    assert any(l.split() and l.split()[0] == "MPI_ABORT" for l in cp.stderr.splitlines())


def _children(pid):
    out = subprocess.run(["ps", "-o", "pid=,stat=,args=", "--ppid", str(pid)], capture_output=True, text=True).stdout
    return [l.split(None, 2) for l in out.splitlines() if l.strip()]


@pytest.mark.parametrize("seed", range(4))
def test_random_external_kill_never_wrong(hostsim, oracle, seed):
    """kill_procs.sh-style: SIGKILL one running rank at a random time.  The job either
    recovers with the right checksum (dead rank's data included) or aborts cleanly; it
    never prints a wrong result and never hangs."""
    rng = random.Random(seed)
    n = rng.choice([5, 9])
    count = 1 << 22
    env = dict(os.environ, FTAR_HOSTSIM_TAG=f"ext{seed}")
    env.pop("FTAR_KILL", None)
    p = subprocess.Popen([os.path.join(hostsim, "bin", "ftrun"), "-np", str(n),
                          os.path.join(hostsim, "src", "raben", "main"), str(count)],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    time.sleep(rng.uniform(0.05, 0.4))
    kids = [c for c in _children(p.pid) if "main" in c[2]]
    if kids:
        victim = int(rng.choice(kids)[0])
        try:
            os.kill(victim, signal.SIGKILL)
        except ProcessLookupError:
            pass  # the rank had already finished: a no-fault run, checked the same way
    out, err = p.communicate(timeout=120)
    hello = {int(l.split()[2]): int(l.split()[-1]) for l in out.splitlines() if l.startswith("Hello")}
    aborted = any(l.split() and l.split()[0] == "MPI_ABORT" for l in err.splitlines())
    assert aborted or set(hello.values()) <= {oracle.expected_checksum(n, count)}
    if not aborted:
        assert len(hello) >= n - 1
    subprocess.run(f"rm -f /dev/shm/ftarhs-ext{seed}-*", shell=True)


RELAY_ALL = {"FTAR_RELAY_MIN": "0", "FTAR_MESH": "0"}  # the step-by-step schedule, relayed


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [3, 4, 5, 6, 8, 9])
def test_relay_nofault_parity(hostsim, oracle, algo, p):
    """Exchanges striped over 2-hop relays give bit-identical results."""
    o, r = _cmp(_fn(oracle, algo), algo, oracle.random_inputs(p, 5003, seed=p), env=RELAY_ALL)
    relayed = [st[0][8] for st in r.status.values()]
    nrecv = p if algo == "raben" and p & (p - 1) == 0 else (1 << (p.bit_length() - 1))
    if nrecv >= 3:
        assert min(relayed) > 0, relayed


@pytest.mark.parametrize("algo,p", [("raben", 5), ("raben", 8), ("raben", 9), ("rd", 4), ("rd", 8), ("rd", 6)])
def test_relay_single_kill_sweep(hostsim, oracle, algo, p):
    """Relays that die before or after forwarding, partners that die mid-step: same
    outcomes and bits as the oracle (lost stripes are re-pulled before the handler)."""
    ins = oracle.random_inputs(p, 3001, seed=p + 1)
    fn = _fn(oracle, algo)
    phases = [1, 2] if algo == "raben" else [1]
    n = 0
    for v in range(p):
        for ph in phases:
            for st in range(3):
                for pt in range(4):
                    ks = [(v, ph, st, pt)]
                    if fn(ins, ks).status[v] != oracle.DEAD:
                        continue
                    _cmp(fn, algo, ins, ks, env=RELAY_ALL)
                    n += 1
    assert n > 0


@pytest.mark.parametrize("seed", range(6))
def test_relay_multi_kill_random(hostsim, oracle, seed):
    rng = random.Random(100 + seed)
    algo = rng.choice(["raben", "rd"])
    p = rng.choice([6, 7, 9, 11])
    victims = rng.sample(range(p), rng.choice([1, 2]))
    kills = [(v, rng.choice([1, 2]) if algo == "raben" else 1, rng.randrange(3), rng.randrange(4)) for v in victims]
    _cmp(_fn(oracle, algo), algo, oracle.random_inputs(p, 2049, seed=seed), kills, env=RELAY_ALL)


CE = {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0", "FTAR_MESH": "0"}


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [2, 3, 4, 5, 8, 9])
def test_copy_engine_nofault_parity(hostsim, oracle, algo, p):
    """Direct pulls as runtime copies + a local reduce over the staged window."""
    _cmp(_fn(oracle, algo), algo, oracle.random_inputs(p, 4099, seed=p + 7), env=CE)


@pytest.mark.parametrize("algo,p", [("raben", 8), ("raben", 9), ("rd", 8), ("rd", 6)])
def test_copy_engine_single_kill_sweep(hostsim, oracle, algo, p):
    ins = oracle.random_inputs(p, 1031, seed=p + 3)
    fn = _fn(oracle, algo)
    phases = [1, 2] if algo == "raben" else [1]
    n = 0
    for v in range(p):
        for ph in phases:
            for st in range(3):
                for pt in (2, 3):  # BARRIER, DURING (copies in flight)
                    ks = [(v, ph, st, pt)]
                    if fn(ins, ks).status[v] != oracle.DEAD:
                        continue
                    _cmp(fn, algo, ins, ks, env=CE)
                    n += 1
    assert n > 0


@pytest.mark.parametrize("p", [2, 4, 8])
def test_raben_redundancy_always_pow2(hostsim, oracle, p):
    """FTAR_REDUNDANCY=1 keeps the reference's step-0 full exchange at power-of-two p,
    where the build skips the half no handler can use: same results and outcomes."""
    ins = oracle.random_inputs(p, 2053, seed=p + 11)
    env = {"FTAR_REDUNDANCY": "1"}
    _cmp(oracle.rabenseifner, "raben", ins, env=env)
    for v in range(p):
        for ph, st in ((1, 0), (1, 1), (2, 0)):
            ks = [(v, ph, st, 2)]
            if oracle.rabenseifner(ins, ks).status[v] == oracle.DEAD:
                _cmp(oracle.rabenseifner, "raben", ins, ks, env=env)


@pytest.mark.parametrize("algo,p", [("rd", 12), ("rd", 16), ("rd", 24), ("rd", 32), ("raben", 17), ("raben", 33),
                                    ("raben", 60), ("raben", 64), ("rd", 64)])
def test_campaign_sizes(hostsim, oracle, algo, p):
    """The reference's fault-campaign N (data/data_fault: RD 4..32, Raben 5..60) and
    the 64-rank maximum: no-fault parity plus single kills at seeded points."""
    fn = _fn(oracle, algo)
    ins = oracle.random_inputs(p, 1031, seed=p + 90)
    _cmp(fn, algo, ins)
    rng = random.Random(p)
    steps = p.bit_length() - 1
    for _ in range(3):
        k = (rng.randrange(p), rng.choice([1, 2]) if algo == "raben" else 1, rng.randrange(steps), 2)
        _cmp(fn, algo, ins, [k])


DEVICE_MODES = {"plain": {}, "inplace": {"FTAR_PROBE_INPLACE": "1"}, "offset1": {"FTAR_PROBE_OFFSET": "1"},
                "inplace_offset3": {"FTAR_PROBE_INPLACE": "1", "FTAR_PROBE_OFFSET": "3"}}


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [1, 2, 4, 5, 8])
@pytest.mark.parametrize("mode", sorted(DEVICE_MODES))
@pytest.mark.parametrize("relay", [False, True])
def test_device_entry_points(hostsim, oracle, algo, p, mode, relay):
    """The device-pointer entry points (what bench.py and torch callers use) on the
    caller's own buffers: in place (sbuf == rbuf), buffers not co-aligned with the
    workspace, two calls per job; sbuf is never written (the probe checks it).  At
    power-of-two p Raben reads sbuf and writes rbuf in place (fast_io)."""
    env = dict(DEVICE_MODES[mode], FTAR_PROBE_DEVICE="1")
    if relay:
        env.update(FTAR_RELAY_MIN="0", FTAR_MESH="0")
    ins = oracle.random_inputs(p, 1031, seed=p + 80)
    o = _fn(oracle, algo)(ins)
    r = H.run_probe(algo, ins, iters=2, backend="hostsim", env_extra=env)
    assert r.returncode == 0, r.stderr[-1000:]
    for w in range(p):
        for it in range(2):
            assert r.status[w][it][0] == 0, (w, it, r.status[w][it])
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


ONESHOT = {"mesh": "0", "oneshot": str(1 << 20), "push": "0", "push2": "0"}  # FTAR_ONESHOT_MAX


def _form_env(form):
    """The mesh's forms: two launches (pull), one-shot, the push reduce-scatter, and push in
    both phases (the owner's tree also stores its block into every peer)."""
    return {"FTAR_ONESHOT_MAX": ONESHOT[form], "FTAR_PUSH": {"push": "1", "push2": "2"}.get(form, "0"),
            "FTAR_MESH_WAIT": "1"}


def _mesh_launches(p, form):
    return 1 if form == "oneshot" and p <= 8 else 2  # FTAR_ONESHOT_MAX=0 turns the one-shot off at p = 2 too


@pytest.mark.parametrize("form", sorted(ONESHOT))
@pytest.mark.parametrize("p", [2, 4, 8, 16])
@pytest.mark.parametrize("dtype,op", [(np.float32, 0), (np.int32, 0), (np.int64, 1), (np.float64, 2), (np.float32, 3)])
def test_mesh_parity(hostsim, oracle, p, dtype, op, form):
    """One-hop reduce-scatter + allgather (power of two, no spare), and its one-shot
    form (every block in its owner's tree, one launch): bit-identical to the step-by-step
    schedule of the oracle for every op, NaN / signed-zero operand order included."""
    ins = oracle.random_inputs(p, 4099, seed=p * 10 + op, dtype=dtype)
    if op >= 2:
        ins = H.with_specials(ins, p + op)
    o, r = _cmp(oracle.rabenseifner, "raben", ins, op=op, env=_form_env(form))
    assert all(st[0][9] == _mesh_launches(p, form) for st in r.status.values()), r.status
    if form.startswith("push"):  # the push forms take their own path: one agree more than the pull form's
        _, rp = _cmp(oracle.rabenseifner, "raben", ins, op=op, env=dict(_form_env("mesh"), FTAR_MESH_WAIT="0"))
        assert all(r.status[w][0][7] == rp.status[w][0][7] + 1 for w in r.status), (r.status, rp.status)
    if form == "mesh":  # the allgather ordered on the device (the default): one agree round fewer
        _, rh = _cmp(oracle.rabenseifner, "raben", ins, op=op, env=dict(_form_env("mesh"), FTAR_MESH_WAIT="0"))
        assert all(r.status[w][0][7] == rh.status[w][0][7] - 1 for w in r.status), (r.status, rh.status)
        assert all(st[0][15] == 1 and st[0][16] == 0 for st in r.status.values()), r.status  # peer_waits, skips
        assert all(st[0][15] == 0 for st in rh.status.values()), rh.status


@pytest.mark.parametrize("p,late", [(4, 3), (8, 0), (2, 1)])
def test_mesh_peer_wait_timeout_fallback(hostsim, oracle, p, late):
    """FTAR_OPT_MESH_WAIT: a rank publishes its tree's flag late (test hook) and its peers'
    device waits give up (FTAR_GATE_TIMEOUT_MS): every rank learns the verdicts in the last
    agree round alike, the ranks whose allgather returned untouched launch it again and one
    more round follows -- same bits as the oracle, two calls, no hang."""
    ins = oracle.random_inputs(p, 40003, seed=p + 61)
    env = dict(_form_env("mesh"), FTAR_GATE_TIMEOUT_MS="30",
               FTAR_PROBE_RANK_ENV=f"{late}:FTAR_PEER_WAIT_DELAY_US=300000")
    o, r = _cmp(oracle.rabenseifner, "raben", ins, env=env)
    for w, st in r.status.items():
        assert st[0][15] == 1, st  # a peer wait every call
        assert st[0][16] == (0 if w == late else 1), (w, st)  # only the others gave up
    ref = H.run_probe("raben", ins, backend="hostsim", env_extra=_form_env("mesh"))
    assert all(r.status[w][0][7] == ref.status[w][0][7] + 1 for w in r.status)  # the extra round, uniform


def test_mesh_peer_wait_off_with_flag_sync_off(hostsim, oracle):
    """FTAR_FLAG_SYNC=0 (fenced-marker drains only, the conservative mode exact_on_node falls
    back to) also keeps the mesh's allgather after a host agree: no peer wait, same bits."""
    ins = oracle.random_inputs(4, 40003, seed=66)
    o, r = _cmp(oracle.rabenseifner, "raben", ins, env=dict(_form_env("mesh"), FTAR_FLAG_SYNC="0"))
    assert all(st[0][15] == 0 for st in r.status.values()), r.status


@pytest.mark.parametrize("kill", [(2, 1, 0, 0), (1, 1, 1, 3), (3, 1, 0, 3), (0, 2, 1, 0), (2, 2, 0, 3), (1, 1, 0, 1)])
def test_mesh_peer_wait_kills_abort(hostsim, oracle, kill):
    """Kills around the device wait at p = 4 (no idle rank: every failure aborts, as the
    reference): before the tree, with the tree in flight before the flag (the peers' waits are
    given up by their failure detectors), during the allgather, after it -- an abort each
    time, never a hang or a result."""
    ins = oracle.random_inputs(4, 40003, seed=sum(kill))
    o = oracle.rabenseifner(ins, [kill])
    assert o.aborted
    r = H.run_probe("raben", ins, [kill], backend="hostsim", timeout=60, env_extra=_form_env("mesh"))
    assert r.aborted and not r.outputs, r.stderr[-1500:]


@pytest.mark.parametrize("form", sorted(ONESHOT))
@pytest.mark.parametrize("p", [4, 8])
def test_mesh_single_kill_sweep(hostsim, oracle, p, form):
    """Every kill point of every step lands in the collapsed phases: the job aborts
    exactly where the reference aborts (all of them, no idle rank)."""
    ins = oracle.random_inputs(p, 1031, seed=p + 500)
    env = _form_env(form)
    n = 0
    for v in range(p):
        for ph in (0, 1, 2, 3):
            for st in range(3):
                for pt in range(4):
                    ks = [(v, ph, st, pt)]
                    if oracle.rabenseifner(ins, ks).status[v] != oracle.DEAD:
                        continue
                    _cmp(oracle.rabenseifner, "raben", ins, ks, env=env)
                    n += 1
    assert n > 0


@pytest.mark.parametrize("form", sorted(ONESHOT))
@pytest.mark.parametrize("p", [2, 8, 16])
@pytest.mark.parametrize("n", [1, 3, 17])
def test_mesh_tiny_counts(hostsim, oracle, p, n, form):
    """Vectors shorter than the rank count: empty final blocks on some ranks (in place:
    the one-shot form stages the input whole)."""
    o, r = _cmp(oracle.rabenseifner, "raben", oracle.random_inputs(p, n, seed=p + n),
                env=dict(_form_env(form), FTAR_PROBE_DEVICE="1", FTAR_PROBE_INPLACE="1"))
    assert all(st[0][9] == _mesh_launches(p, form) for st in r.status.values())


@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("mode", sorted(DEVICE_MODES))
def test_oneshot_device_buffers(hostsim, oracle, p, mode):
    """One-shot mesh on the caller's device buffers (in place, misaligned), two calls:
    exact, sbuf never written, one launch per call; above the threshold the two-launch
    mesh runs."""
    ins = oracle.random_inputs(p, 1031, seed=p + 960)
    o = oracle.rabenseifner(ins)
    for limit, launches in ((str(1 << 20), 1), ("1024", 1 if p == 2 else 2)):  # p = 2: one-shot at any size
        env = dict(DEVICE_MODES[mode], FTAR_PROBE_DEVICE="1", FTAR_ONESHOT_MAX=limit)
        r = H.run_probe("raben", ins, iters=2, backend="hostsim", env_extra=env)
        assert r.returncode == 0, r.stderr[-1000:]
        for w in range(p):
            for it in range(2):
                assert r.status[w][it][0] == 0, (w, it, r.status[w][it])
                assert r.status[w][it][9] == launches, (limit, r.status[w][it])
                assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("gate", ["1", "0"])
def test_gated_launches(hostsim, oracle, algo, p, gate):
    """Small calls at a power of two queue their exchange launches ahead of the barrier
    that readies the operands, behind a gate (FTAR_GATE, default on): Raben's one-shot
    launch (one per call), every RD step's (log2 p per call: step 0 behind the staging
    copy, step s + 1 behind step s); none replaced, same bits.  FTAR_GATE=0 launches after
    the barriers."""
    ins = oracle.random_inputs(p, 1031, seed=p + 970)
    o = _fn(oracle, algo)(ins)
    r = H.run_probe(algo, ins, iters=3, backend="hostsim", env_extra={"FTAR_GATE": gate, "FTAR_GATE_HOLD_US": "0"})
    assert r.returncode == 0, r.stderr[-1000:]
    per_call = (1 if algo == "raben" else p.bit_length() - 1) if gate == "1" else 0
    for w in range(p):
        for it in range(3):
            assert r.status[w][it][0] == 0, r.status[w][it]
            assert algo == "rd" or r.status[w][it][9] == 1, r.status[w][it]
            assert r.status[w][it][10:12] == (per_call, 0), r.status[w][it]
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("algo,p", [("rd", 2), ("rd", 4), ("rd", 8)])
def test_gated_launches_mid_size(hostsim, oracle, algo, p):
    """Mid-size vectors (1 MiB < S <= FTAR_GATE_MAX, set to 16 MiB -- the default is 1 MiB, see
    DESIGN.md 6; here 2 MiB + 12 B, read in place, not staged): RD queues steps 1.. ahead of their barriers (step 0 reads the peers'
    inputs, whose mappings are known after the first barrier only); none replaced, same bits.
    Above FTAR_GATE_MAX nothing is gated.  (The mesh's allgather is ordered on the device
    instead: test_device_wait_at_the_headline_size.)"""
    n = (1 << 19) + 3
    ins = oracle.random_inputs(p, n, seed=p + 990)
    o = _fn(oracle, algo)(ins)
    env = {"FTAR_GATE_HOLD_US": "0", "FTAR_RELAY": "0", "FTAR_HOSTSIM_PINNED": "1", "FTAR_GATE_MAX": str(16 << 20)}
    r = H.run_probe(algo, ins, iters=2, backend="hostsim", env_extra=env)
    assert r.returncode == 0, r.stderr[-1000:]
    per_call = p.bit_length() - 2
    for w in range(p):
        for it in range(2):
            assert r.status[w][it][10:12] == (per_call, 0), (w, it, r.status[w][it])
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)
    r = H.run_probe(algo, ins, backend="hostsim", env_extra=dict(env, FTAR_GATE_MAX=str(1 << 20)))
    assert r.returncode == 0 and all(r.status[w][0][10] == 0 for w in range(p)), r.status


@pytest.mark.timeout(300)
def test_device_wait_at_the_headline_size(hostsim):
    """The mesh at the headline size (256 MiB float32-sized vectors, here int32 so the sum is
    exact in any order): its allgather is ordered behind the peers' trees on the device -- one
    peer wait per call, none given up, nothing queued behind a host gate even with
    FTAR_GATE_MAX >= S (the gated-allgather form of round 4 is gone), the result exact."""
    p, n = 4, 1 << 26
    rng = np.random.default_rng(11)
    ins = [rng.integers(-1 << 20, 1 << 20, n, dtype=np.int32) for _ in range(p)]
    want = np.sum(np.stack(ins), axis=0, dtype=np.int64).astype(np.int32)
    env = {"FTAR_GATE_HOLD_US": "0", "FTAR_PROBE_DEVICE": "1", **H.MESH_FORM, "FTAR_GATE_MAX": str(4 * n)}
    r = H.run_probe("raben", ins, iters=2, backend="hostsim", env_extra=env, timeout=280)
    assert r.returncode == 0, r.stderr[-1000:]
    for w in range(p):
        for it in range(2):
            st = r.status[w][it]
            assert st[9] == 2 and st[10] == 0 and st[15] == 1 and st[16] == 0, (w, it, st)
            assert np.array_equal(r.outputs[w][it], want), (w, it)


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [2, 4])
def test_gated_launch_replaced_when_a_peer_reads_in_place(hostsim, oracle, algo, p):
    """A peer that lets its send buffer be read in place (here: its own FTAR_STAGE_MAX=0)
    moves its input away from the staged IN a gated launch was planned on: after the
    inputs are resolved the plans differ, the gated launch is skipped (returns untouched)
    and a fresh one runs -- same bits."""
    ins = oracle.random_inputs(p, 1031, seed=p + 980)
    o = _fn(oracle, algo)(ins)
    env = {"FTAR_PROBE_RANK_ENV": "1:FTAR_STAGE_MAX=0",  # host entry: sbuf = the exportable staging
           "FTAR_GATE_HOLD_US": "0"}  # (a loaded test host must not give gates up: the counts are checked)
    r = H.run_probe(algo, ins, iters=2, backend="hostsim", env_extra=env)
    assert r.returncode == 0, r.stderr[-1000:]
    L = p.bit_length() - 1
    for w in range(p):
        for it in range(2):
            st = r.status[w][it]
            assert st[0] == 0, st
            # rank 1 stages nothing: no gate for its one-shot / its RD step 0 (whose operands
            # it cannot predict), RD steps 1.. still gated (they read accumulators).  Raben:
            # every other rank's one-shot reads rank 1's input -> replaced.  RD: only rank 0
            # reads rank 1's input (its step-0 partner)
            if w == 1:
                want = (0, 0) if algo == "raben" else (L - 1, 0)
            elif algo == "raben":
                want = (1, 1)
            else:
                want = (L, 1 if w == 0 else 0)
            assert st[10:12] == want, (w, st)
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("p", [2, 4])
@pytest.mark.parametrize("mesh", ["1", "0"])
def test_host_pipeline_chunks(hostsim, oracle, p, mesh):
    """Host buffers of >= 16 MiB at power-of-two p go through as a pipeline of chunk
    Allreduces (H2D / Allreduce / D2H overlapped): same bits as one call."""
    _cmp(oracle.rabenseifner, "raben", oracle.random_inputs(p, (1 << 22) + 77, seed=p + 900), env={"FTAR_MESH": mesh})


@pytest.mark.parametrize("algo,p", [("raben", 4), ("rd", 4), ("raben", 8), ("rd", 6)])
def test_peer_input_map_failure_falls_back(hostsim, oracle, algo, p):
    """A rank that cannot map a peer's exported send buffer: the extra agree round of the
    call turns exporting off everywhere, the exporters stage their inputs, and the call
    (and the next) are still exact."""
    ins = oracle.random_inputs(p, 5003, seed=p + 950)
    o = _fn(oracle, algo)(ins)
    r = H.run_probe(algo, ins, iters=2, backend="hostsim",
                    env_extra={"FTAR_HOSTSIM_FAIL_IMPORT": str(4 * (p - 1) + 1), "FTAR_STAGE_MAX": "0"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "inputs are staged from now on" in r.stderr
    for w in range(p):
        for it in range(2):
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("p", [2, 4])
@pytest.mark.parametrize("op", [2, 3])
def test_host_pipeline_operand_order(hostsim, oracle, p, op):
    """MAX/MIN on floats depend on the operand order (NaN, signed zeros), and the order
    of an element's tree depends on the block that owns it: a chunk pipeline would move
    block boundaries, so a float MAX/MIN host call >= 16 MiB must stay one call."""
    ins = oracle.random_inputs(p, (1 << 22) + 77, seed=p + 40 * op)
    rng = np.random.default_rng(p + op)
    for x in ins:
        k = rng.integers(0, x.size, 1 << 16)
        x[k[: 1 << 15]] = np.nan
        x[k[1 << 15:]] = rng.choice(np.array([0.0, -0.0], dtype=np.float32), 1 << 15)
    _cmp(oracle.rabenseifner, "raben", ins, op=op)


SPECIAL_TRANSPORTS = {
    "default": {},
    "relay": RELAY_ALL,
    "direct": {"FTAR_RELAY": "0", "FTAR_MESH": "0"},
    "direct_serial": {"FTAR_RELAY": "0", "FTAR_MESH": "0", "FTAR_OVERLAP": "0"},
    "copy_engine": CE,
    "reference_shape": {"FTAR_RELAY": "0", "FTAR_MESH": "0", "FTAR_OVERLAP": "0", "FTAR_REDUNDANCY": "1"},
}


@pytest.mark.parametrize("transport", sorted(SPECIAL_TRANSPORTS))
@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [2, 3, 5, 8, 9])
def test_operand_order_specials(hostsim, oracle, transport, algo, p):
    """MAX/MIN on floats with NaN and signed zeros pin the operand order of every
    combination -- for both schedules, spare layouts (p = 3, 5, 9) and every transport,
    not only the mesh."""
    for op, dt in ((2, np.float32), (3, np.float64)):
        ins = H.with_specials(oracle.random_inputs(p, 4099, seed=p * 13 + op, dtype=dt), p + 7 * op)
        _cmp(_fn(oracle, algo), algo, ins, op=op, env=dict(SPECIAL_TRANSPORTS[transport], FTAR_RELAY_MIN="0")
             if transport != "default" else None)


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p,op", [(5, 2), (6, 3), (9, 2)])
def test_operand_order_specials_recovery(hostsim, oracle, algo, p, op):
    """The recovery paths (impersonation replay, spare promotion, RD block selection)
    keep the operand order too: every kill point the oracle recovers from, MAX/MIN with
    NaN / signed zeros / infinities, bit-exact on every survivor."""
    ins = H.with_specials(oracle.random_inputs(p, 1031, seed=p + 77), p + 3)
    fn = _fn(oracle, algo)
    n = 0
    for v in range(p):
        for ph in range(4):
            for st in range(3):
                for pt in range(4):
                    o = fn(ins, [(v, ph, st, pt)], op=op)
                    if o.aborted or oracle.DEAD not in o.status:
                        continue
                    _cmp(fn, algo, ins, [(v, ph, st, pt)], op=op)
                    n += 1
    assert n > 0


@pytest.mark.parametrize("seed", range(4))
def test_raben_two_failures_random(hostsim, oracle, seed):
    """Two failures at different steps (p = 11, three idle spares): the first recovery's
    new entry must hold the dead rank's whole reduce-scatter state, because the second
    recovery's replay pulls its sindex windows of earlier steps.  It held only the
    current window and the result lost a block's contributions (SUM 40 instead of 55)."""
    import random
    rnd = random.Random(seed)
    p = 11
    pts = [(v, ph, st, pt) for v in range(p) for ph in (1, 2) for st in range(3) for pt in range(4)]
    ins = H.with_specials(oracle.random_inputs(p, 1031, seed=p + seed), p + seed)
    n = 0
    for ks in [((4, 1, 1, 2), (0, 1, 2, 1)), ((8, 1, 2, 0), (10, 1, 1, 0))] + [tuple(rnd.sample(pts, 2))
                                                                            for _ in range(60)]:
        if ks[0][0] == ks[1][0]:
            continue
        for op in (0, 2):
            o = oracle.rabenseifner(ins, list(ks), op=op)
            if o.aborted or sum(st == oracle.DEAD for st in o.status) < 2:
                continue
            _cmp(oracle.rabenseifner, "raben", ins, list(ks), op=op)
            n += 1
    assert n > 0


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("ks", [((1, 1, 2, 2), (6, 1, 2, 2)), ((8, 1, 2, 2), (6, 1, 2, 2)), ((3, 1, 1, 2), (9, 1, 1, 2))])
def test_two_barrier_victims_same_step(hostsim, oracle, algo, ks):
    """Two ranks killed at the same step's BARRIER point: each waits for the others to
    finish the step, but not for the other victim (they used to wait for each other
    forever); the job then recovers or aborts like the oracle."""
    p = 11
    ins = H.with_specials(oracle.random_inputs(p, 1031, seed=p + 78), p + 4)
    for op in (0, 2):
        _cmp(_fn(oracle, algo), algo, ins, list(ks), op=op)


def test_staging_allocation_failure_aborts_job(hostsim, oracle):
    """A rank whose pinned staging allocation fails (the _host entry points) ends the job
    with MPI_Abort instead of returning alone while its peers wait in the collective;
    nothing is left half-allocated for a later call to run into."""
    ins = oracle.random_inputs(4, 1031, seed=41)
    r = H.run_probe("raben", ins, iters=2, backend="hostsim", timeout=60,
                    env_extra={"FTAR_HOSTSIM_FAIL_PLAIN": "1", "FTAR_HOSTSIM_FAIL_RANK": "2"})
    assert r.aborted, r.stderr[-1000:]
    assert "staging allocation" in r.stderr and r.returncode == 102, (r.returncode, r.stderr[-1000:])
    assert not r.outputs


@pytest.mark.parametrize("which", ["raben", "rd"])
def test_shm_exhaustion_is_nomem_abort(hostsim, which):
    """Host-sim "device memory" that runs out (here a deliberately tiny budget; in a container
    whose /dev/shm is full, posix_fallocate's ENOSPC) is an allocation error: the job ends with
    MPI_Abort and FTAR_ERR_NOMEM (102), naming the allocation -- not a SIGBUS at the first touch
    that the job would report as a rank death, errorcode 75."""
    cp, hello = H.run_driver(which, 4, 1 << 20, env_extra={"FTAR_HOSTSIM_SHM_BUDGET": str(1 << 20)}, timeout=60)
    out = cp.stdout + cp.stderr
    assert "with errorcode 102" in out and "errorcode 75" not in out, out[-1500:]
    assert "out of shared memory" in out
    assert not hello


@pytest.mark.parametrize("algo,count,fail", [
    ("raben", 1031, "2:h2d:0"), ("raben", 1031, "1:d2h:0"), ("rd", 1031, "3:h2d:0"), ("rd", 1031, "0:d2h:0"),
    # >= 16 MiB at p = 4: the chunk pipeline (two 8 MiB chunk Allreduces); the failing copy is
    # the second chunk's H2D (queued before the first chunk's Allreduce) or the second D2H
    ("raben", (1 << 22) + 77, "2:h2d:1"), ("raben", (1 << 22) + 77, "1:d2h:1")])
def test_host_copy_failure_aborts_job(hostsim, oracle, algo, count, fail):
    """A rank-local H2D / D2H failure inside a _host entry point ends the job (MPI_Abort with
    FTAR_ERR_DEVICE) instead of returning alone while the peers spin in the next barrier
    (VERDICT r05 next #2): every rank gone well inside the timeout, and an MPI_ABORT line
    that check_fault.py classifies as ABORT."""
    import time
    ins = oracle.random_inputs(4, count, seed=43)
    t0 = time.time()
    r = H.run_probe(algo, ins, iters=2, backend="hostsim", timeout=60, env_extra={"FTAR_HOSTSIM_FAIL_COPY": fail})
    assert time.time() - t0 < 50
    assert r.returncode == 101, (r.returncode, r.stderr[-1500:])
    assert any(l.startswith("MPI_ABORT") for l in r.stderr.splitlines()), r.stderr[-1500:]
    assert "copy failed: injected" in r.stderr
    assert f"rank {fail.split(':')[0]}: " in r.stderr
    assert not any(len(v) == 2 for v in r.outputs.values())  # no rank finished both calls


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_torchrun_bootstrap(hostsim, oracle, tmp_path, algo):
    """ftar_init's torchrun branch (RANK / WORLD_SIZE / MASTER_PORT, no ftrun): the
    control block is named after the port and the elastic agent's pid, rank 0 creates
    it -- the bootstrap bench.py uses at N > 1.  Two ranks, bit-exact to the oracle."""
    import sys
    import socket
    p = 2
    ins = oracle.random_inputs(p, 4099, seed=77)
    for r_, x in enumerate(ins):
        x.tofile(str(tmp_path / f"in_{r_}.bin"))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, FTAR_PROBE_DIR=str(tmp_path), FTAR_PROBE_ALGO=algo, FTAR_PROBE_DTYPE="1",
               FTAR_PROBE_COUNT=str(ins[0].size), FTAR_HOSTSIM_TAG=f"tr{os.getpid()}", OMP_NUM_THREADS="1")
    for k in ("FTAR_JOB", "FTAR_RANK", "FTAR_SIZE", "FTAR_LAUNCHER", "FTAR_KILL"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={p}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "--no-python",
           os.path.join(hostsim, "bin", "ftar_probe")]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    subprocess.run(f"rm -f /dev/shm/ftarhs-tr{os.getpid()}-*", shell=True)
    assert cp.returncode == 0, cp.stderr[-2000:]
    o = oracle.rabenseifner(ins) if algo == "raben" else oracle.recursive_doubling(ins)
    for r_ in range(p):
        got = np.fromfile(str(tmp_path / f"out_{r_}_0.bin"), dtype=np.float32)
        assert np.array_equal(got.view(np.uint32), o.outputs[r_].view(np.uint32)), r_
        st = open(tmp_path / f"status_{r_}_0.txt").read().split()
        assert st[0] == "0" and st[2] == str(p), st


from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

TRANSPORTS = [{}, {"FTAR_RELAY_MIN": "0", "FTAR_MESH": "0"}, {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0"},
              {"FTAR_MESH": "0", "FTAR_RELAY": "0", "FTAR_OVERLAP": "0"}, {"FTAR_EXPORT": "0"},
              {"FTAR_ONESHOT_MAX": "0"}, {"FTAR_REDUNDANCY": "1", "FTAR_MESH": "0"}]


@settings(max_examples=int(os.environ.get("FTAR_PROPERTY_EXAMPLES", "120")), deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(algo=st.sampled_from(["raben", "rd"]), p=st.integers(1, 13), count=st.integers(1, 3000),
       dtype=st.sampled_from([np.float32, np.int32, np.int64, np.float64]), op=st.integers(0, 9),
       transport=st.integers(0, len(TRANSPORTS) - 1), kill=st.none() | st.tuples(
           st.integers(0, 12), st.integers(0, 3), st.integers(0, 3), st.integers(0, 3)),
       seed=st.integers(0, 10 ** 6))
def test_property_any_shape_transport_kill(hostsim, oracle, algo, p, count, dtype, op, transport, kill, seed):
    """Any rank count, ragged length, dtype, op, transport and (optionally) one kill point:
    the outcome class and every survivor's bits equal the oracle's (floats carry NaN /
    signed zeros / infinities, so MAX / MIN pin the operand order; integers also take
    MPI's logical / bitwise ops, on inputs with zeros)."""
    if op >= 4 and dtype in (np.float32, np.float64):
        op %= 4  # logical / bitwise ops exist for the integer types only (MPI_ERR_OP)
    ins = oracle.random_inputs(p, count, seed=seed, dtype=dtype)
    if dtype in (np.float32, np.float64):
        ins = H.with_specials(ins, p + 2)
    elif op in (4, 6, 8):
        for x in ins:
            x[::3] = 0
    kills = []
    if kill is not None and kill[0] < p:
        kills = [kill]
        o = _fn(oracle, algo)(ins, kills, op=op)
        if not o.aborted and o.status[kill[0]] != oracle.DEAD:
            kills = []  # a point this schedule never reaches at this p
    _cmp(_fn(oracle, algo), algo, ins, kills, op=op, env=TRANSPORTS[transport])


@settings(max_examples=int(os.environ.get("FTAR_PROPERTY_EXAMPLES", "120")) // 2, deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(algo=st.sampled_from(["raben", "rd"]), p=st.integers(2, 13), count=st.integers(1, 2000),
       dtype=st.sampled_from([np.float32, np.int32]), op=st.integers(0, 3),
       transport=st.integers(0, len(TRANSPORTS) - 1), iters=st.integers(1, 3),
       kills=st.lists(st.tuples(st.integers(0, 12), st.integers(0, 3), st.integers(0, 3), st.integers(0, 3)),
                      max_size=3, unique_by=lambda k: k[0]),
       seed=st.integers(0, 10 ** 6))
def test_property_multi_kill_repeated_calls(hostsim, oracle, algo, p, count, dtype, op, transport, iters, kills,
                                            seed):
    """Up to three deaths in the first call, then more calls on the re-targeted comm:
    call 0 as the oracle's faulty run, every later call as the oracle's fault-free run
    over the survivors in their new order."""
    fn = _fn(oracle, algo)
    ins = oracle.random_inputs(p, count, seed=seed, dtype=dtype)
    if dtype == np.float32:
        ins = H.with_specials(ins, p + 2)
    ks = [k for k in kills if k[0] < p]
    while True:  # keep the kill points call 0 reaches (an unreached one would fire in a later call)
        o1 = fn(ins, ks, op=op)
        if o1.aborted:
            break
        reached = [k for k in ks if o1.status[k[0]] == O.DEAD]
        if reached == ks:
            break
        ks = reached
    if all(s == O.DEAD for s in o1.status):
        return
    r = H.run_probe(algo, ins, ks, op=op, iters=iters, backend="hostsim", timeout=120, env_extra=TRANSPORTS[transport])
    if o1.aborted:
        assert r.aborted and not r.outputs, (ks, r.stderr[-1000:])
        return
    assert not r.aborted and r.returncode == 0, (ks, r.stderr[-1000:])
    u = {4: np.uint32, 8: np.uint64}[ins[0].dtype.itemsize]
    o2 = fn([ins[w] for w in o1.order_after], op=op) if iters > 1 else None
    for w, s in enumerate(o1.status):
        if s != 0:
            assert w not in r.outputs
            continue
        assert np.array_equal(r.outputs[w][0].view(u), o1.outputs[w].view(u)), (ks, w)
        for it in range(1, iters):
            i = o1.order_after.index(w)
            assert np.array_equal(r.outputs[w][it].view(u), o2.outputs[i].view(u)), (ks, w, it)


def _bit_inputs(p, n, seed, dt):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(p):
        v = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        v[rng.random(n) < 0.3] = 0
        out.append(v)
    return out


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p,op", [(3, 4), (4, 5), (5, 6), (8, 7), (9, 8), (6, 9), (2, 9), (16, 5)])
def test_nofault_logical_bitwise(hostsim, oracle, algo, p, op):
    """MPI's logical / bitwise ops (integer types) through both schedules, every
    transport's code path the defaults pick (mesh / one-shot at powers of two)."""
    dt = np.int64 if p % 2 else np.int32
    _cmp(_fn(oracle, algo), algo, _bit_inputs(p, 1031, p * 13 + op, dt), op=op)


@pytest.mark.parametrize("algo,p,kill", [("raben", 9, (6, 1, 1, 3)), ("raben", 5, (4, 2, 0, 0)), ("rd", 6, (3, 1, 1, 3)),
                                         ("rd", 8, (5, 1, 0, 1))])
@pytest.mark.parametrize("op", [4, 7, 9])
def test_kill_logical_bitwise(hostsim, oracle, algo, p, kill, op):
    """A recovering kill under a bitwise op: the handlers' replays and re-sends reduce
    with the call's op (not SUM)."""
    _cmp(_fn(oracle, algo), algo, _bit_inputs(p, 777, p + op, np.int32), [kill], op=op)


@pytest.mark.parametrize("p", [5, 9])
def test_withdrawn_dead_input_aborts(hostsim, oracle, p):
    """Without the step-0 redundancy copy (FTAR_REDUNDANCY=0, or the auto default on one GPU),
    the RS replay reads the dead rank's step-0 input where it lies (deviation 6):
    a process death leaves it mapped, a lost device does not.  FTAR_KILL_WITHDRAW makes the
    victim withdraw its input as it dies (its workspace generation moves on, its published
    sbuf is retracted): the replay must then refuse to read it and the job abort -- never a
    result from a stale or unmapped buffer.  With the reference's copy (FTAR_REDUNDANCY=1)
    the same kills recover bit-exact like the oracle, and reduce-scatter kills of the idle
    spare, which need no replay, recover either way."""
    ins = oracle.random_inputs(p, 257, seed=p + 7)
    n_abort = n_rec = 0
    elided = {"FTAR_KILL_WITHDRAW": "1", "FTAR_REDUNDANCY": "0"}
    for v in range(p):
        for st in (1, 2):
            for pt in range(4):
                ks = [(v, 1, st, pt)]
                o = oracle.rabenseifner(ins, ks)
                if o.aborted or o.status[v] != oracle.DEAD:
                    continue
                replay = v != 1  # rank 1 is the idle odd rank of the pre-step pair (rem = 1)
                r = H.run_probe("raben", ins, ks, backend="hostsim", env_extra=elided)
                if replay:
                    assert r.aborted and not r.outputs, (ks, r.stderr[-800:])
                    assert "not readable" in r.stderr, r.stderr[-800:]
                    n_abort += 1
                else:
                    _cmp(oracle.rabenseifner, "raben", ins, ks, env=elided)
                    n_rec += 1
                _cmp(oracle.rabenseifner, "raben", ins, ks, env={"FTAR_KILL_WITHDRAW": "1", "FTAR_REDUNDANCY": "1"})
    assert n_abort > 0 and n_rec > 0, (n_abort, n_rec)


@pytest.mark.parametrize("p", [5, 9])
def test_redundancy_auto_follows_the_devmap(hostsim, oracle, p):
    """FTAR_REDUNDANCY unset (auto): with a spare, the step-0 copy moves when the comm spans
    more than one GPU -- so a replay never depends on a dead process's memory staying
    readable across devices (the reference copies at step 0 because that memory is gone,
    raben/rabenseifner.c:206-211) -- and is elided when every rank shares one GPU (where a
    peer's mapping provably keeps it).  Two-device devmap: every replaying kill recovers
    bit-exact against the oracle even when the victim withdraws its input as it dies; one
    device: the copy is elided (step0_copy 0) and the same withdrawn input aborts."""
    ins = oracle.random_inputs(p, 257, seed=p + 9)
    two = ",".join(str(r % 2) for r in range(p))
    one = ",".join("0" for _ in range(p))
    n = 0
    for v in range(2, p):  # ranks whose death needs the impersonation replay
        ks = [(v, 1, 1, 3)]  # reduce-scatter step 1, mid-exchange
        o = oracle.rabenseifner(ins, ks)
        if o.aborted or o.status[v] != oracle.DEAD:
            continue
        r = H.run_probe("raben", ins, ks, backend="hostsim", devmap=two, env_extra={"FTAR_KILL_WITHDRAW": "1"})
        assert not r.aborted, (ks, r.stderr[-800:])
        for w, s in enumerate(o.status):
            if s == 0:
                assert np.array_equal(r.outputs[w][0].view(np.uint32), o.outputs[w].view(np.uint32)), (ks, w)
                assert r.status[w][0][12] == 1, r.status[w][0]  # the copy moved
        r1 = H.run_probe("raben", ins, ks, backend="hostsim", devmap=one, env_extra={"FTAR_KILL_WITHDRAW": "1"})
        assert r1.aborted and "not readable" in r1.stderr, (ks, r1.stderr[-800:])
        n += 1
    assert n > 0
    r = H.run_probe("raben", ins, backend="hostsim", devmap=one)
    assert all(r.status[w][0][12] == 0 for w in range(p)), r.status
    r = H.run_probe("raben", ins, backend="hostsim", devmap=two)
    assert all(r.status[w][0][12] == 1 for w in range(p)), r.status
    # power of two (no spare): no handler can use the copy, whatever the layout
    r = H.run_probe("raben", ins[:4], backend="hostsim", devmap="0,1,2,3")
    assert all(r.status[w][0][12] == 0 for w in range(4)), r.status


def test_redundancy_auto_uses_physical_device_ids(hostsim, oracle):
    """under per-rank HIP_VISIBLE_DEVICES masks every rank may see its own GPU as
    ordinal 0.  The auto redundancy decision compares the physical identities the ranks
    publish (PCI bus ids; FTAR_HOSTSIM_PHYS stands in for them here), not the ordinals: one
    ordinal on two physical GPUs moves the step-0 copy, and a replaying kill recovers bit-exact
    with the victim's input withdrawn; one physical GPU under every ordinal elides it."""
    p = 5
    ins = oracle.random_inputs(p, 257, seed=41)
    one_ordinal = ",".join("0" for _ in range(p))
    two_phys = ",".join(f"0000:{5 + r % 2:02x}:00.0" for r in range(p))
    r = H.run_probe("raben", ins, backend="hostsim", devmap=one_ordinal, env_extra={"FTAR_HOSTSIM_PHYS": two_phys})
    assert all(r.status[w][0][12] == 1 for w in range(p)), r.status  # the copy moved
    same_phys = ",".join("0000:05:00.0" for _ in range(p))
    r = H.run_probe("raben", ins, backend="hostsim", devmap="0,1,0,1,0", env_extra={"FTAR_HOSTSIM_PHYS": same_phys})
    assert all(r.status[w][0][12] == 0 for w in range(p)), r.status  # one physical GPU: elided
    ks = [(3, 1, 1, 3)]
    o = oracle.rabenseifner(ins, ks)
    assert not o.aborted and o.status[3] == oracle.DEAD
    r = H.run_probe("raben", ins, ks, backend="hostsim", devmap=one_ordinal,
                    env_extra={"FTAR_HOSTSIM_PHYS": two_phys, "FTAR_KILL_WITHDRAW": "1"})
    assert not r.aborted, r.stderr[-800:]
    for w, s in enumerate(o.status):
        if s == 0:
            assert np.array_equal(r.outputs[w][0].view(np.uint32), o.outputs[w].view(np.uint32)), w


def test_node_layout_random_kills_never_read_dead_memory(hostsim):
    """The node's layout (rank r on device r % 8: the auto redundancy moves Raben's step-0
    copy) with every victim withdrawing its memory as it dies (FTAR_KILL_WITHDRAW, a lost
    device): random single and double kills at p = 9 / 11 (Raben with spares) and 6 / 8 (RD)
    recover or abort exactly as the oracle, so no recovery path reads a dead rank's HBM
    (`tests/fault_sweep.py --spread 8 --withdraw` draws thousands; profiles/r05/sweeps)."""
    import random
    import fault_sweep as FS
    rnd = random.Random(5)
    ran = 0
    for _ in range(60):
        algo = rnd.choice(["raben", "rd"])
        p = rnd.choice([9, 11] if algo == "raben" else [6, 8])
        pts = [(v, ph, st, pt) for v in range(p) for ph in (1, 2) for st in range(3) for pt in range(4)]
        ks = tuple(rnd.sample(pts, rnd.choice([1, 2])))
        if len({k[0] for k in ks}) < len(ks):
            continue
        devmap = ",".join(str(r % 8) for r in range(p))
        res = FS.run_one(algo, p, rnd.choice([0, 2, 3]), ks, 257, aborts=True, devmap=devmap,
                         env={"FTAR_KILL_WITHDRAW": "1"})
        if res is None:
            continue
        assert res == "ok", (algo, p, ks, res)
        ran += 1
    assert ran >= 30, ran


def _cycle_run(oracle, algo, p, seq, kills=(), seed=0):
    """FTAR_PROBE_CYCLE_SEQ: call k sends from exportable buffer seq[k] (every buffer holds the
    rank's input); inputs above FTAR_STAGE_MAX=0 are exported where the schedule allows."""
    inputs = oracle.random_inputs(p, 3001, seed=seed)
    env = {"FTAR_PROBE_DEVICE": "1", "FTAR_PROBE_CYCLE_SEQ": ",".join(map(str, seq)), "FTAR_STAGE_MAX": "0",
           "FTAR_VERBOSE": "2"}
    r = H.run_probe(algo, inputs, kills, iters=len(seq), backend="hostsim", timeout=180, env_extra=env)
    assert "not in this rank's cache" not in r.stderr and "failed" not in r.stderr, r.stderr[-3000:]
    return inputs, r


@pytest.mark.parametrize("algo,p", [("raben", 4), ("raben", 6), ("rd", 5), ("rd", 8)])
def test_send_buffer_cycling_mirrored_caches(hostsim, oracle, algo, p):
    """A caller cycling through 12 send buffers, more than the peers' mapping caches hold
    (FTAR_UCACHE = 8): the first 8 are exported and mapped once, the others staged call after
    call -- no mapping is dropped and re-made -- and every one of the 36 results is exact.
    Exporter and importers apply one admission rule to one sequence of allocations, so they
    agree on what is mapped without a message (ftar_comm.c xcache_admit / peer_sbuf)."""
    seq = list(range(12)) * 2 + list(range(11, -1, -1))
    inputs, r = _cycle_run(oracle, algo, p, seq, seed=p + 40)
    assert r.returncode == 0 and not r.aborted, r.stderr[-2000:]
    o = _fn(oracle, algo)(inputs)
    for w in range(p):
        for it in range(len(seq)):
            assert r.status[w][it][0] == 0, (w, it, r.status[w][it])
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)
    # mappings made: one per peer for each allocation admitted, none re-made
    mapped = [line for line in r.stderr.splitlines() if "mapped rank" in line]
    exported_new = [line for line in r.stderr.splitlines() if ", new)" in line]
    per_rank = {w: sum(1 for m in mapped if m.startswith(f"ftar[{w}] ")) for w in range(p)}
    news = {w: sum(1 for m in exported_new if m.startswith(f"ftar[{w}] ")) for w in range(p)}
    # (Raben's pre-step pairs stage their inputs: only the others export)
    assert all(news[w] <= 8 for w in range(p)) and sum(news.values()) >= 8 * (p - 2 * (p - (1 << (p.bit_length() - 1)))), news
    assert all(per_rank[w] == sum(news[u] for u in range(p) if u != w) for w in range(p)), (per_rank, news)


def test_send_buffer_cycling_with_a_kill(hostsim, oracle):
    """A rank dies in call 2 (a call that admits a new buffer); the survivors recover and keep
    cycling on the shrunk comm: the dead rank's mappings are dropped, the caches of the
    survivors stay in agreement, every later result equals the oracle's on the survivors."""
    p, seq = 6, list(range(10)) * 2
    kills = [(4, 1, 1, 2, 2)]
    inputs, r = _cycle_run(oracle, "raben", p, seq, kills=kills, seed=91)
    assert r.returncode == 0 and not r.aborted, r.stderr[-2000:]
    o0 = oracle.rabenseifner(inputs)
    o1 = oracle.rabenseifner(inputs, [k[:4] for k in kills])
    assert not o1.aborted
    order = o1.order_after
    o2 = oracle.rabenseifner([inputs[w] for w in order])
    for i, w in enumerate(order):
        for it in range(len(seq)):
            want = o0.outputs[w] if it < 2 else o1.outputs[w] if it == 2 else o2.outputs[i]
            assert np.array_equal(r.outputs[w][it].view(np.uint32), want.view(np.uint32)), (w, it)
