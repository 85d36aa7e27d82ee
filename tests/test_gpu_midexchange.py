"""Kills with data in flight, and the BASELINE configs at their full size, on the GPU.

FTAR_PT_DURING (include/ftar.h): the victim has entered the step, launched its own pull
kernel, waited until every peer launched its pulls of the step (its partner's kernel
reads the victim's HBM), and is SIGKILLed with its kernel still queued or running.  The
reference's counterpart is a Sendrecv cut short by the death
(/root/reference/src/raben/rabenseifner.c:209-211 returns an error, :238-241 marks the
received window `corr`): the partner discards what it pulled and the error handler
rebuilds the window (raben/errhandler.c:159-181).  The oracle models exactly that, so
survivors must match it bit for bit -- with MAX over NaN / signed zeros the operand
order of the rebuilt window shows that the `corr` path ran.

Full size: BASELINE.json configs[2..4] are 256 MiB of float32 per rank at p = 8 (and
C5: p = 9 = 8 + one idle spare, a kill mid-exchange).  Every rank of these jobs shares
the one GPU of the test box, so the fabric is local HBM; the schedules, IPC mappings,
control plane and recovery are the ones the 8-GPU node runs.
"""
import os

import numpy as np
import pytest

import harness as H

pytestmark = pytest.mark.gpu

ALL_ON_GPU0 = ",".join(["0"] * 16)
FULL = 1 << 26  # 64 Mi float32 = 256 MiB per rank
RELAY_ALL = {"FTAR_RELAY_MIN": "0", "FTAR_MESH": "0"}
REFERENCE_SHAPE = {"FTAR_MESH": "0", "FTAR_REDUNDANCY": "1", "FTAR_OVERLAP": "0", "FTAR_RELAY": "0"}


def _check(fn, algo, inputs, kills=(), op=0, env=None, timeout=300):
    o = fn(inputs, kills, op=op)
    # the withdrawal hook lives only in the TEST-ONLY hooks build of the library
    backend = "gpu_hooks" if env and "FTAR_KILL_WITHDRAW" in env else "gpu"
    r = H.run_probe(algo, inputs, kills, op=op, backend=backend, devmap=ALL_ON_GPU0, timeout=timeout,
                    env_extra=env)
    u = {4: np.uint32, 8: np.uint64}[inputs[0].dtype.itemsize]
    if o.aborted:
        assert r.aborted, r.stderr[-2000:]
        assert not r.outputs
        return o, r
    assert not r.aborted, r.stderr[-2000:]
    assert r.returncode == 0, r.stderr[-2000:]
    for w, st in enumerate(o.status):
        if st == 0:
            assert w in r.outputs, (w, r.stderr[-2000:])
            assert np.array_equal(r.outputs[w][0].view(u), o.outputs[w].view(u)), (w, algo, kills)
        else:
            assert w not in r.outputs
    return o, r


def _died_mid_exchange(r, victim):
    """The victim's own line: 'rank V dies mid-exchange (...): own kernel X, N peers launched'."""
    for line in r.stderr.splitlines():
        if f"rank {victim} dies mid-exchange" in line:
            t = line.split(":")[-1].split(",")
            return "in flight" in t[0], int(t[1].split()[0])
    raise AssertionError(f"no mid-exchange death of rank {victim}: {r.stderr[-2000:]}")


# C5 layout: 9 ranks = 8 + idle spare (rank 1 pairs with rank 0 in the pre-step); the
# victim original rank 6 is vrank 5
@pytest.mark.parametrize("kill", [(6, 1, 1, 3), (6, 2, 1, 3), (3, 1, 2, 3), (8, 2, 0, 3), (6, 1, 0, 3),
                                  (6, 2, 2, 3), (0, 1, 1, 3), (1, 1, 1, 3)])
def test_during_kill_p9(oracle, kill):
    """RS step 1 / AG step 1 / RS step 2 / last AG step recover (new_entry = the spare);
    RS step 0 and the first AG step abort (raben/errhandler.c:37-38, 320-323); the
    spare's partner and the idle spare itself die mid-exchange."""
    o, r = _check(oracle.rabenseifner, "raben", oracle.random_inputs(9, (1 << 20) + 5, seed=90 + kill[0]), [kill])
    if not o.aborted:
        assert r.status and all(st[0][3] == 1 for w, st in r.status.items()), r.status  # one recovery
    _died_mid_exchange(r, kill[0])


@pytest.mark.parametrize("kill", [(3, 1, 1, 3), (2, 1, 1, 3), (4, 1, 1, 3)])
def test_during_kill_p5_operand_order(oracle, kill):
    """p = 5 (4 + one idle spare), MAX over NaN / signed zeros / infinities: the partner's
    window must be the handler's rebuild (impersonator's operand order), not the pull."""
    ins = H.with_specials(oracle.random_inputs(5, 65536 + 5, seed=500 + kill[0]), 11)
    o = oracle.rabenseifner(ins, [kill], op=2)
    assert not o.aborted and o.status[kill[0]] == oracle.DEAD
    _check(oracle.rabenseifner, "raben", ins, [kill], op=2)


@pytest.mark.parametrize("form", ["0", str(1 << 20)])
@pytest.mark.parametrize("kill", [(3, 1, 1, 3), (5, 2, 0, 3), (0, 1, 2, 3)])
def test_during_kill_mesh_p8_aborts(oracle, kill, form):
    """p = 8, no idle rank: the one-hop mesh (two-launch and one-shot) with a rank dying
    while every peer's tree kernel reads its send buffer -- the job aborts like the
    reference (new_entry = -1, raben/errhandler.c:207-211)."""
    o, r = _check(oracle.rabenseifner, "raben", oracle.random_inputs(8, (1 << 18) + 3, seed=kill[0]), [kill],
                  env={"FTAR_ONESHOT_MAX": form})
    assert o.aborted


@pytest.mark.parametrize("algo,p,kill,env", [("raben", 9, (6, 1, 1, 3), RELAY_ALL), ("raben", 9, (4, 2, 1, 3), RELAY_ALL),
                                             ("rd", 8, (2, 1, 1, 3), RELAY_ALL), ("rd", 8, (5, 1, 2, 3), None),
                                             ("rd", 6, (1, 1, 1, 3), None), ("raben", 9, (6, 1, 1, 3),
                                                                             {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0"})])
def test_during_kill_transports(oracle, algo, p, kill, env):
    """Mid-exchange deaths under the 2-hop relay (the victim is also a relay of other
    receivers' stripes), the copy-engine transport, and recursive doubling (shrink branch
    at p = 8, spare branch at p = 6)."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    _check(fn, algo, oracle.random_inputs(p, (1 << 20) + 7, seed=p * 10 + kill[0]), [kill], env=env)


# ---- BASELINE configs at full size ---------------------------------------------------

@pytest.mark.timeout(900)
def test_full_size_c3_rd_p8(oracle):
    """configs[2]: recursive doubling, 256 MiB float32 SUM, 8 ranks."""
    _check(oracle.recursive_doubling, "rd", oracle.random_inputs(8, FULL, seed=703), timeout=600)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("shape", ["mesh", "reference"] + H.wide("push", "push2"))
def test_full_size_c4_raben_p8(oracle, shape):
    """configs[3]: Rabenseifner, 256 MiB float32 SUM, 8 ranks -- the default one-hop
    mesh, its push form, and the reference's shape (step by step, pairwise, step-0 full
    exchange)."""
    # one device-resident 256 MiB call per rank (no host-pipeline chunking)
    env = dict(REFERENCE_SHAPE if shape == "reference" else dict(H.MESH_FORM, FTAR_PUSH={"push": "1", "push2": "2"}
                                                                  .get(shape, "0")), FTAR_HOST_PIPE="0")
    o, r = _check(oracle.rabenseifner, "raben", oracle.random_inputs(8, FULL, seed=704), env=env, timeout=600)
    mesh_steps = {st[0][9] for st in r.status.values()}
    assert mesh_steps == ({0} if shape == "reference" else {2}), r.status


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("kill", [(6, 1, 1, 3), (6, 2, 1, 3)])
def test_full_size_c5_p9_kill_mid_exchange(oracle, kill):
    """configs[4]: Rabenseifner, 256 MiB float32 SUM, 9 ranks (8 + idle spare), vrank 5
    killed in reduce-scatter step 1 with its own 64 MiB pull kernel in flight and its
    partner's pull reading its HBM -- and, as SURVEY.md 8d also asks, in allgather step 1
    (a middle AG step): recovered, bit-exact to the oracle."""
    o, r = _check(oracle.rabenseifner, "raben", oracle.random_inputs(9, FULL, seed=705), [kill], timeout=900,
                  env={"FTAR_VERBOSE": "1"})
    assert not o.aborted and o.recoveries == 1
    in_flight, peers = _died_mid_exchange(r, 6)
    assert peers >= 1
    print(f"victim kernel in flight: {in_flight}, peers launched: {peers}")
    if kill[1] == 1:
        assert "died mid-exchange at RS step 1" in r.stderr, r.stderr[-2000:]


@pytest.mark.timeout(900)
def test_full_size_mesh_p8_kill_mid_exchange_aborts(oracle):
    """p = 8 at 256 MiB: a rank dies while the seven peers' tree kernels read its 256 MiB
    send buffer over the mesh -- a clean abort, no hang, no device fault."""
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(8, FULL, seed=706), [(5, 1, 0, 3)], timeout=600)


def _seeds(var, default):
    """Seeds of the random GPU kill tests; FTAR_GPU_KILL_SEEDS / FTAR_GPU_KILL2_SEEDS
    ("2,3,4" or "2-11") widen a one-off campaign without editing the suite."""
    v = os.environ.get(var)
    if not v:
        return default
    if "-" in v:
        a, b = v.split("-")
        return list(range(int(a), int(b) + 1))
    return [int(t) for t in v.split(",")]


KILL_COUNTS = [int(c) for c in os.environ.get("FTAR_GPU_KILL_COUNTS", "").split(",") if c]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed,count", [(s, c) for s in _seeds("FTAR_GPU_KILL_SEEDS", [0] + H.wide(1))
                                        for c in (KILL_COUNTS or [(1 << 20) + 3])] +
                         ([] if KILL_COUNTS else [(0, 1031)]))
def test_random_kill_points_gpu(oracle, seed, count):
    """Random single kills (any victim, phase, step and point -- DURING weighted up) on
    the GPU, p = 5 / 9 (one idle spare) and 6 / 8, both schedules, 1 Mi elements (and 1031:
    the small calls, whose launches wait behind gates -- a victim may die with its gated
    launch queued), MAX over NaN / signed zeros so the recovery path shows in the bits:
    outcome class and every survivor's result as the oracle's.  Twelve jobs per seed, each a
    real process teardown, most with a peer's kernel reading the victim's HBM (six per seed
    by default, twelve under FTAR_GPU_WIDE=1).
    FTAR_GPU_KILL_COUNTS ("1031,65536") sets the lengths of a one-off campaign."""
    import random
    rng = random.Random(seed)
    n = 0
    while n < (12 if H.WIDE else 6):
        algo = rng.choice(["raben", "rd"])
        p = rng.choice([5, 9] if algo == "raben" else [6, 8, 9])
        kill = (rng.randrange(p), rng.choice([1, 2]) if algo == "raben" else 1, rng.randrange(3),
                rng.choice([3, 3, 0, 1, 2]))
        fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
        ins = H.with_specials(oracle.random_inputs(p, count, seed=seed * 100 + n), p)
        if fn(ins, [kill], op=2).status[kill[0]] != oracle.DEAD:
            continue  # the schedule never reaches this point (e.g. a step it does not have)
        _check(fn, algo, ins, [kill], op=2)
        n += 1


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", _seeds("FTAR_GPU_KILL2_SEEDS", [0]))
def test_random_two_kills_gpu(oracle, seed):
    """Two deaths in one call on the GPU (distinct victims, any phase / step / point,
    mid-exchange weighted up): Raben p = 9 / 11 (one / three idle spares), RD p = 6 / 8,
    MAX over NaN / signed zeros; outcome class and every survivor's bits as the oracle's
    (the host-sim sweep tests/fault_sweep.py draws the same cases by the thousand)."""
    import random
    rng = random.Random(1000 + seed)
    n = 0
    while n < (6 if H.WIDE else 3):
        algo = rng.choice(["raben", "rd"])
        p = rng.choice([9, 11] if algo == "raben" else [6, 8])
        pts = [(v, ph, st, pt) for v in range(p) for ph in ((1, 2) if algo == "raben" else (1,))
               for st in range(3) for pt in (3, 3, 0, 1, 2)]
        kills = rng.sample(pts, 2)
        if kills[0][0] == kills[1][0]:
            continue
        fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
        ins = H.with_specials(oracle.random_inputs(p, (1 << 18) + 3, seed=seed * 100 + n), p)
        o = fn(ins, kills, op=2)
        if sum(st == oracle.DEAD for st in o.status) < 2 and not o.aborted:
            continue  # a point the schedule never reaches
        _check(fn, algo, ins, kills, op=2)
        n += 1


# The node's recovery shape: ranks on 8 GPUs make the auto redundancy move Raben's step-0
# copy (FTAR_REDUNDANCY=1 here, where every rank shares GPU 0), and a victim's HBM may go
# with it (FTAR_KILL_WITHDRAW: its workspace generation moves on and its send buffer is
# retracted, so any plan that would read it refuses).  On one GPU a dead process's mapping
# stays readable, so only this makes a recovery that still reads it fail here.
NODE_SHAPE = {"FTAR_REDUNDANCY": "1", "FTAR_KILL_WITHDRAW": "1"}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("algo,p,kill", [("raben", 9, (6, 1, 1, 3)), ("raben", 9, (3, 1, 2, 3)),
                                         ("raben", 9, (6, 2, 1, 3)), ("raben", 9, (8, 2, 0, 3)),
                                         ("raben", 5, (3, 1, 1, 3)), ("rd", 6, (1, 1, 1, 3)),
                                         ("rd", 8, (5, 1, 2, 3))])
def test_node_shape_recovery_reads_no_dead_memory(oracle, algo, p, kill):
    """Recoveries in the node's shape (step-0 copy moved, the victim's memory withdrawn as it
    dies): RS steps 1 / 2 replayed from the partner's copy, AG kills served by the original
    partner, RD's shrink and spare branches -- bit-exact against the oracle (MAX over NaN /
    signed zeros pins the recovery path), none refused for a dead rank's input (the host-sim
    draws thousands of these: tests/fault_sweep.py --spread 8 --withdraw)."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    ins = H.with_specials(oracle.random_inputs(p, (1 << 20) + 3, seed=800 + kill[0]), p)
    o, r = _check(fn, algo, ins, [kill], op=2, env=NODE_SHAPE)
    assert not o.aborted and o.status[kill[0]] == oracle.DEAD
    assert "withdraws its input" in r.stderr and "not readable" not in r.stderr, r.stderr[-1500:]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", _seeds("FTAR_GPU_NODE_SHAPE_SEEDS", [0]))
def test_node_shape_random_kills(oracle, seed):
    """Random single and double kills in the node's shape (NODE_SHAPE), Raben p = 5 / 9 / 11
    and RD p = 6 / 8: outcome class and every survivor's bits as the oracle's."""
    import random
    rng = random.Random(2000 + seed)
    n = 0
    while n < (8 if H.WIDE else 4):
        algo = rng.choice(["raben", "rd"])
        p = rng.choice([5, 9, 11] if algo == "raben" else [6, 8])
        pts = [(v, ph, st, pt) for v in range(p) for ph in ((1, 2) if algo == "raben" else (1,))
               for st in range(3) for pt in (3, 3, 0, 1, 2)]
        kills = rng.sample(pts, rng.choice([1, 2]))
        if len({k[0] for k in kills}) < len(kills):
            continue
        fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
        ins = H.with_specials(oracle.random_inputs(p, (1 << 18) + 3, seed=seed * 100 + n), p)
        o = fn(ins, kills, op=2)
        if o.aborted or sum(st == oracle.DEAD for st in o.status) < len(kills):
            continue  # recoveries only: an abort shows nothing about the memory they read
        _check(fn, algo, ins, kills, op=2, env=NODE_SHAPE)
        n += 1


from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

GPU_TRANSPORTS = [{}, {"FTAR_RELAY_MIN": "0", "FTAR_MESH": "0"}, {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0"},
                  {"FTAR_EXPORT": "0"}, {"FTAR_ONESHOT_MAX": "0"}, {"FTAR_REDUNDANCY": "1", "FTAR_MESH": "0"}]


@pytest.mark.timeout(900)
@settings(max_examples=int(os.environ.get("FTAR_GPU_PROPERTY_EXAMPLES", "20" if H.WIDE else "10")), deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture], database=None)
@given(algo=st.sampled_from(["raben", "rd"]), p=st.integers(2, 8), count=st.integers(1, 300000),
       op=st.integers(0, 3), transport=st.integers(0, len(GPU_TRANSPORTS) - 1), iters=st.integers(1, 2),
       kills=st.lists(st.tuples(st.integers(0, 7), st.integers(0, 3), st.integers(0, 3), st.integers(0, 3)),
                      max_size=2, unique_by=lambda k: k[0]),
       seed=st.integers(0, 10 ** 6))
def test_property_gpu(oracle, algo, p, count, op, transport, iters, kills, seed):
    """The host-sim property test on the GPU: any rank count 2-8, ragged length up to
    300k float32 (NaN / signed zeros / infinities), op, transport and up to two kill
    points in call 0, then a second call on the re-targeted comm; outcome and bits as the
    oracle's."""
    import oracle as O
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    ins = H.with_specials(oracle.random_inputs(p, count, seed=seed), p + 2)
    ks = [k for k in kills if k[0] < p]
    while True:
        o1 = fn(ins, ks, op=op)
        if o1.aborted:
            break
        reached = [k for k in ks if o1.status[k[0]] == O.DEAD]
        if reached == ks:
            break
        ks = reached
    r = H.run_probe(algo, ins, ks, op=op, iters=iters, backend="gpu", devmap=ALL_ON_GPU0, timeout=300,
                    env_extra=GPU_TRANSPORTS[transport])
    if o1.aborted:
        assert r.aborted and not r.outputs, (ks, r.stderr[-2000:])
        return
    assert not r.aborted and r.returncode == 0, (ks, r.stderr[-2000:])
    o2 = fn([ins[w] for w in o1.order_after], op=op) if iters > 1 else None
    for w, s in enumerate(o1.status):
        if s != 0:
            assert w not in r.outputs
            continue
        assert _same(r.outputs[w][0], o1.outputs[w], op), (ks, w)
        for it in range(1, iters):
            i = o1.order_after.index(w)
            assert _same(r.outputs[w][it], o2.outputs[i], op), (ks, w, it)


def _same(got, want, op):
    """Bit equality; for SUM / PROD a NaN matches any NaN.  When both operands of an add
    or multiply are NaN, IEEE 754 (6.2.3) leaves open which payload (and sign) the result
    carries, and compilers swap the operands of commutative ops freely -- the oracle's gcc
    and the kernels' hipcc pick differently (inf + -inf then NaN + NaN).  MAX / MIN select
    an operand and stay bit-exact."""
    if op >= 2:
        return np.array_equal(got.view(np.uint32), want.view(np.uint32))
    gn, wn = np.isnan(got), np.isnan(want)
    return np.array_equal(gn, wn) and np.array_equal(got[~gn].view(np.uint32), want[~wn].view(np.uint32))
