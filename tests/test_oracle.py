"""The CPU oracle pinned against the reference's own recorded results.

Golden data (tests/golden/, extracted by make_golden.py from the reference's data/ CSVs):
  * ref_checksums.csv: the per-rank checksum sum_i(result[i] % 17) printed by the
    reference drivers for int32 SUM with buffer[i] = rank, NP in {4..64}, every recorded SIZE
    (1 .. 2^27).
  * ref_fault_outcomes.csv: outcomes of the reference's random single-kill campaign.
"""
import csv
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _wrap32(v):
    return (v + 2**31) % 2**32 - 2**31


def load_checksums():
    with open(os.path.join(GOLDEN, "ref_checksums.csv")) as f:
        return [(r["algo"], int(r["NP"]), int(r["SIZE"]), int(r["RESULT"])) for r in csv.DictReader(f, delimiter=";")]


def test_golden_rows_present():
    rows = load_checksums()
    assert len(rows) > 500
    assert {r[1] for r in rows} >= {4, 6, 8, 12, 16, 24, 32, 48, 64}


@pytest.mark.parametrize("algo", ["rd", "raben"])
def test_checksums_match_reference(oracle, algo):
    """Every recorded (NP, SIZE) checksum of the reference is reproduced by the oracle's
    schedule (both FT algorithms and the vendor baselines record the same values)."""
    fn = oracle.recursive_doubling if algo == "rd" else oracle.rabenseifner
    rows = [r for r in load_checksums() if r[0] in (algo, "original_" + algo)]
    by_np = {}
    for _, np_, size, res in rows:
        by_np.setdefault(np_, []).append((size, res))
    for np_, items in by_np.items():
        # results are constant vectors: simulate a small count fully, then check the
        # recorded checksum for every recorded SIZE (and the full checksum for small ones)
        small = [s for s, _ in items if s <= 64]
        cnt = max(small) if small else 64
        r = fn(oracle.rank_inputs(np_, cnt))
        assert not r.aborted
        v = int(r.outputs[0][0])
        for w in range(np_):
            assert (r.outputs[w] == v).all()
        for size, res in items:
            assert _wrap32((v % 17) * size) == res, (algo, np_, size)
            if size <= cnt:
                assert oracle.checksum17(r.outputs[np_ - 1][:size]) == res


@pytest.mark.parametrize("algo,np_", [("rd", 4), ("rd", 6), ("raben", 5), ("raben", 9)])
def test_full_checksum_simulation(oracle, algo, np_):
    fn = oracle.recursive_doubling if algo == "rd" else oracle.rabenseifner
    for size in (1, 7, 1000, 16384):
        r = fn(oracle.rank_inputs(np_, size))
        for w in range(np_):
            assert oracle.checksum17(r.outputs[w]) == oracle.expected_checksum(np_, size)


def load_fault_outcomes():
    with open(os.path.join(GOLDEN, "ref_fault_outcomes.csv")) as f:
        return [dict(algo=r["algo"], N=int(r["N"]), killed=int(r["KILLED"]), abort=r["ABORT"] == "True",
                     deadlock=r["DEADLOCK"] == "True", right=r["RIGHT"] == "True", count=int(r["count"]))
                for r in csv.DictReader(f, delimiter=";")]


def _single_kill_outcomes(oracle, algo, n, count=8):
    fn = oracle.recursive_doubling if algo == "rd" else oracle.rabenseifner
    ins = oracle.rank_inputs(n, count)
    phases = [oracle.PH_LOOP] if algo == "rd" else [oracle.PH_LOOP, oracle.PH_AG]
    outcomes = []
    for v in range(n):
        for ph in phases:
            for st in range(6):
                r = fn(ins, [(v, ph, st, oracle.PT_BEFORE)])
                if r.status[v] != oracle.DEAD:
                    continue
                ok = (not r.aborted and all(oracle.checksum17(r.outputs[w]) == oracle.expected_checksum(n, count)
                                            for w in range(n) if r.status[w] == oracle.OK))
                outcomes.append(("abort" if r.aborted else ("right" if ok else "wrong"), v, ph, st, r))
    return outcomes


@pytest.mark.parametrize("algo,n", [("rd", 4), ("rd", 8), ("rd", 16), ("raben", 5), ("raben", 9), ("raben", 17)])
def test_fault_outcomes_match_reference_campaign(oracle, algo, n):
    """The reference recorded, for this N, single-kill runs that recovered with the right
    result and runs that aborted; the oracle reproduces both classes and never computes
    a wrong result."""
    rows = [r for r in load_fault_outcomes() if r["algo"] == algo and r["N"] == n]
    recovered = sum(r["count"] for r in rows if r["killed"] == 1 and r["right"] and not r["abort"]
                    and not r["deadlock"])
    aborted = sum(r["count"] for r in rows if r["abort"])
    assert recovered > 0 and aborted > 0
    kinds = [o[0] for o in _single_kill_outcomes(oracle, algo, n)]
    assert "right" in kinds and "abort" in kinds
    assert "wrong" not in kinds


def test_rd_pow2_recovery_rule(oracle):
    """rd/errhandler.c: a death in the first step always aborts (check_abort, util.c:49-78:
    the dead rank and its partner form a lost block); later deaths shrink and recover."""
    for n in (4, 8, 16):
        for kind, v, ph, st, r in _single_kill_outcomes(oracle, "rd", n):
            assert kind == ("abort" if st == 0 else "right"), (n, v, st)


def test_raben_recovery_rules(oracle):
    """raben/errhandler.c: abort on a reduce-scatter step-0 death (:37-38), on a death in
    the first allgather step (:320-323), or when no idle rank is left (:210-211)."""
    for n in (4, 8, 16):  # power of two: no idle rank
        assert all(o[0] == "abort" for o in _single_kill_outcomes(oracle, "raben", n))
    for n in (5, 9, 17):
        steps = int(np.log2(n))
        for kind, v, ph, st, r in _single_kill_outcomes(oracle, "raben", n):
            if ph == oracle.PH_LOOP:
                assert kind == ("abort" if st == 0 else "right"), (n, v, st)
            else:
                assert kind == ("abort" if st == steps - 1 else "right"), (n, v, st)


def test_rd_nonpow2_deviation_recovers(oracle):
    """The reference deadlocks here (rd/errhandler.c:100-111 never advances j); the
    restatement recovers with the spare and flags the deviation."""
    r = oracle.recursive_doubling(oracle.rank_inputs(6, 32), [(1, oracle.PH_LOOP, 1, oracle.PT_BEFORE)])
    assert not r.aborted and r.deviations & 0x1
    for w in range(6):
        if w != 1:
            assert oracle.checksum17(r.outputs[w]) == oracle.expected_checksum(6, 32)


def _tree(vals):
    while len(vals) > 1:
        vals = [vals[i] + vals[i + 1] for i in range(0, len(vals), 2)]
    return vals[0]


def test_float_reduction_tree(oracle):
    """With p = 2^L both schedules reduce every element as a balanced binary tree in
    rank order; with a pre-step the pairs (2i, 2i+1) are added first."""
    for p in (2, 4, 8, 16):
        ins = oracle.random_inputs(p, 4097, seed=p)
        want = _tree(list(ins)).view(np.uint32)
        for fn in (oracle.rabenseifner, oracle.recursive_doubling):
            r = fn(ins)
            for w in range(p):
                assert (r.outputs[w].view(np.uint32) == want).all()
    ins = oracle.random_inputs(6, 1001, seed=6)  # Raben: rem=2, vranks {0+1, 2+3, 4, 5}
    want = _tree([ins[0] + ins[1], ins[2] + ins[3], ins[4], ins[5]]).view(np.uint32)
    r = oracle.rabenseifner(ins)
    assert all((r.outputs[w].view(np.uint32) == want).all() for w in range(6))
    ins = oracle.random_inputs(6, 1001, seed=7)  # RD: active 0..3, inactive 4,5 fold into 0,1
    want = _tree([ins[0] + ins[4], ins[1] + ins[5], ins[2], ins[3]]).view(np.uint32)
    r = oracle.recursive_doubling(ins)
    assert all((r.outputs[w].view(np.uint32) == want).all() for w in range(6))


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.int64, np.float64])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_reduce_local_semantics(oracle, dt, op):
    rng = np.random.default_rng(3)
    a = (rng.integers(-1000, 1000, 999)).astype(dt)
    b = (rng.integers(-1000, 1000, 999)).astype(dt)
    inout = b.copy()
    oracle.reduce_local(a, inout, op)
    want = {0: b + a, 1: b * a, 2: np.where(b > a, b, a), 3: np.where(b < a, b, a)}[op]
    assert (inout == want.astype(dt)).all()


def test_int32_wraparound(oracle):
    x = [np.full(5, 2**31 - 1, np.int32), np.full(5, 1, np.int32)]
    r = oracle.rabenseifner(x)
    assert (r.outputs[0] == np.int32(-2**31)).all()


def test_zero_count(oracle):
    r = oracle.rabenseifner([np.zeros(0, np.int32)] * 4)
    assert r.ret == 14  # MPI_ERR_UNKNOWN from copy_buffer (raben/util.c:40-43)


def test_reference_wrong_result_rows_are_harness_artefacts(oracle):
    """The reference's campaign recorded RIGHT RESULT=False rows (data/data_fault, e.g.
    log_single_Raben.csv `17;2.0;110124421;1;...;False`).  They are not recovery
    failures: as many occur in runs where no rank died (KILLED=0: every rank printed its
    Hello line, so no failure and no error handler ran and the schedule is deterministic)
    -- 43 of 51 for RD, 8 of 21 for Raben -- at no lower a rate than with a kill, and
    concentrated at N >= 24 where 4 N stdout lines of concurrently printing ranks pass
    through one mpiexec output stream (check_fault.py:70-88 parses them).  For every
    such N the schedule itself (the oracle, no fault) produces the reference's closed-form
    checksum."""
    rows = load_fault_outcomes()
    for algo in ("rd", "raben"):
        wrong = [r for r in rows if r["algo"] == algo and not r["right"]]
        nokill = sum(r["count"] for r in wrong if r["killed"] == 0)
        assert nokill >= 8 and nokill / sum(r["count"] for r in wrong) > 0.3
        fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
        for n in sorted({r["N"] for r in wrong}):
            o = fn(oracle.rank_inputs(n, 257))
            assert all(oracle.checksum17(x) == oracle.expected_checksum(n, 257) for x in o.outputs), (algo, n)


# MPI's logical and bitwise predefined ops (include/ftar.h): numpy restatements
BIT_OPS = {4: lambda b, a: ((b != 0) & (a != 0)), 5: lambda b, a: b & a, 6: lambda b, a: ((b != 0) | (a != 0)),
           7: lambda b, a: b | a, 8: lambda b, a: ((b != 0) ^ (a != 0)), 9: lambda b, a: b ^ a}


def bit_inputs(p, n, seed, dt):
    """Integers with many zeros (the logical ops) and full-width bit patterns (the bitwise ones)."""
    rng = np.random.default_rng(seed)
    out = []
    for r in range(p):
        v = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        v[rng.random(n) < 0.3] = 0
        out.append(v)
    return out


@pytest.mark.parametrize("dt", [np.int32, np.int64])
@pytest.mark.parametrize("op", [4, 5, 6, 7, 8, 9])
def test_reduce_local_logical_bitwise(oracle, dt, op):
    a, b = bit_inputs(2, 4099, op, dt)
    inout = b.copy()
    oracle.reduce_local(a, inout, op)
    assert (inout == BIT_OPS[op](b, a).astype(dt)).all()


@pytest.mark.parametrize("op", [4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_logical_bitwise_on_float_is_err_op(oracle, op, dt):
    """MPI_ERR_OP (9) for a logical / bitwise op on a floating-point type, in the local
    reduce and in both schedules; unknown ops are MPI_ERR_ARG."""
    a = np.ones(8, dt)
    b = np.ones(8, dt)
    rc = oracle.lib().ftar_oracle_reduce_local(oracle.DTYPE_OF[a.dtype], op, a.ctypes.data, b.ctypes.data, 8)
    assert rc == 9
    assert oracle.rabenseifner([a, b], op=op).ret == 9
    assert oracle.recursive_doubling([a, b], op=op).ret == 9
    assert oracle.rabenseifner([a, b], op=10).ret == 13


@pytest.mark.parametrize("algo", ["rd", "raben"])
@pytest.mark.parametrize("p", [2, 3, 5, 8, 9])
@pytest.mark.parametrize("op", [4, 5, 6, 7, 8, 9])
def test_schedules_logical_bitwise(oracle, algo, p, op):
    """Every rank ends with the fold of all inputs (these ops commute and associate
    exactly, so any schedule order gives the numpy fold)."""
    from functools import reduce
    dt = np.int64 if op % 2 else np.int32
    ins = bit_inputs(p, 1031, p * 10 + op, dt)
    want = reduce(lambda acc, x: BIT_OPS[op](acc, x).astype(dt), ins[1:], ins[0])
    r = (oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling)(ins, op=op)
    assert r.ret == 0
    for w in range(p):
        assert (r.outputs[w] == want).all(), w
