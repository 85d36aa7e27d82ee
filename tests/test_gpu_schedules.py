"""GPU parity of the two fault-tolerant schedules against the CPU oracle.

Each case launches P rank processes with ftrun (all on GPU 0 of the one-GPU test box:
the IPC peer mappings, pull kernels, control plane and recovery run exactly as on 8
GPUs, only the fabric is local HBM) and compares every survivor's output bit for bit
with the oracle's global simulation of the reference on the same inputs.  Kill cases
use deterministic injection (FTAR_KILL) and check both the outcome class (recover vs
MPI_Abort) and the data.
"""
import os

import numpy as np
import pytest

import harness as H

pytestmark = pytest.mark.gpu

ALL_ON_GPU0 = ",".join(["0"] * 16)


def _check(oracle_fn, algo, inputs, kills=(), op=0, iters=1, env=None):
    o = oracle_fn(inputs, kills, op=op)
    r = H.run_probe(algo, inputs, kills, op=op, iters=iters, backend="gpu", devmap=ALL_ON_GPU0, timeout=300,
                    env_extra=env)
    u = {4: np.uint32, 8: np.uint64}[inputs[0].dtype.itemsize]
    if o.aborted:
        assert r.aborted, r.stderr[-2000:]
        assert not r.outputs
        return o, r
    assert not r.aborted, r.stderr[-2000:]
    for w, st in enumerate(o.status):
        if st == 0:
            assert w in r.outputs, (w, r.stderr[-2000:])
            got = r.outputs[w][0]
            assert np.array_equal(got.view(u), o.outputs[w].view(u)), (w, algo, kills)
        else:
            assert w not in r.outputs
    return o, r


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 8, 9])
def test_schedule_nofault_float32(oracle, algo, p):
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    _check(fn, algo, oracle.random_inputs(p, 100003, seed=p))


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float64])
def test_schedule_nofault_dtypes(oracle, algo, dtype):
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    _check(fn, algo, oracle.random_inputs(6, 4099, seed=3, dtype=dtype))


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_schedule_reference_inputs_checksum(oracle, algo):
    """The reference drivers' case: buffer[i] = rank, int32 SUM, checksum closed form."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    o, r = _check(fn, algo, oracle.rank_inputs(8, 16384))
    for w in range(8):
        assert oracle.checksum17(r.outputs[w][0]) == oracle.expected_checksum(8, 16384)


@pytest.mark.parametrize("kill", [(5, 1, 1, 2), (5, 1, 2, 2), (1, 1, 1, 2), (4, 2, 1, 2), (3, 2, 0, 2),
                                  (6, 1, 0, 2), (2, 2, 2, 2), (5, 1, 1, 0), (7, 2, 1, 1)])
def test_raben_single_kill_p9(oracle, kill):
    """C5 layout: 9 ranks = 8 + one idle spare (rank 1); recoverable and aborting cases."""
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(9, 65536 + 5, seed=9), [kill])


@pytest.mark.parametrize("kill", [(3, 1, 1, 2), (0, 1, 2, 2), (2, 1, 0, 2), (6, 1, 1, 0), (5, 1, 2, 1)])
def test_rd_single_kill(oracle, kill):
    p = 8 if kill[0] < 8 else 9
    _check(oracle.recursive_doubling, "rd", oracle.random_inputs(p, 65536 + 3, seed=4), [kill])


RECOVERING_P5 = [("raben", k) for k in [(0, 1, 1, 0), (4, 1, 1, 1), (0, 2, 0, 0), (4, 2, 0, 1), (3, 1, 1, 3),
                                         (2, 2, 0, 3)] + H.wide((3, 1, 1, 0), (2, 1, 1, 1))] + \
                [("rd", k) for k in [(0, 1, 1, 0), (4, 1, 1, 1), (1, 1, 1, 3), (0, 1, 1, 2)] +
                 H.wide((3, 1, 1, 0), (2, 1, 1, 1), (4, 1, 0, 3), (3, 1, 1, 3))]


@pytest.mark.parametrize("algo,kill", RECOVERING_P5)
def test_kill_operand_order_specials(oracle, algo, kill):
    """A partner's exchange failed iff the victim died before completing it (exchange
    entry / completion tokens in the control block), not whenever its death was noticed:
    with MAX over NaN / signed zeros / infinities the replayed state's operand order shows
    which path ran, so survivors must match the oracle bit for bit (p = 5: 4 + one idle
    spare).  Every listed point recovers (recursive doubling has no allgather phase)."""
    p = 5
    ins = H.with_specials(oracle.random_inputs(p, 65536 + 5, seed=p + 77), p + 3)
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    o = fn(ins, [kill], op=2)
    assert not o.aborted and o.status[kill[0]] == oracle.DEAD
    _check(fn, algo, ins, [kill], op=2)


def test_rd_spare_branch_p6(oracle):
    """Non power of two: an active death is repaired by waking the spare (deviation from
    the reference, which spins forever at rd/errhandler.c:100-111)."""
    _check(oracle.recursive_doubling, "rd", oracle.random_inputs(6, 10007, seed=6), [(1, 1, 1, 2)])


def test_raben_two_failures_p11(oracle):
    """Two sequential recoveries (rem = 3 idle ranks)."""
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(11, 30011, seed=11), [(4, 1, 1, 2), (9, 2, 1, 2)])


def test_repeated_calls_after_recovery(oracle):
    """The comm is re-targeted by a recovery and the next call runs on the survivors."""
    inputs = oracle.random_inputs(5, 20000, seed=2)
    r = H.run_probe("raben", inputs, [(3, 1, 1, 2)], iters=3, backend="gpu", devmap=ALL_ON_GPU0)
    o1 = oracle.rabenseifner(inputs, [(3, 1, 1, 2)])
    assert not r.aborted, r.stderr[-2000:]
    survivors = [w for w in range(5) if w != 3]
    for w in survivors:
        assert np.array_equal(r.outputs[w][0].view(np.uint32), o1.outputs[w].view(np.uint32))
        assert r.status[w][1][2] == 4  # comm size after the recovery
    # later calls: a 4-rank comm in the re-targeted order; the sum is over survivors
    order = o1.order_after
    o2 = oracle.rabenseifner([inputs[w] for w in order])
    for i, w in enumerate(order):
        for it in (1, 2):
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o2.outputs[i].view(np.uint32))


def test_driver_checksums(oracle):
    """The drop-in src/raben/main and src/rd/main print the reference's lines."""
    for which in ("raben", "rd"):
        cp, hello = H.run_driver(which, 4, 100000, backend="gpu", env_extra={"FTAR_DEVMAP": ALL_ON_GPU0})
        assert cp.returncode == 0, cp.stderr[-2000:]
        assert sorted(hello) == [0, 1, 2, 3]
        assert set(hello.values()) == {oracle.expected_checksum(4, 100000)}
        assert "P: 4" in cp.stdout and "Size: 100000" in cp.stdout and "Time:" in cp.stdout


def _golden_checksums():
    import csv
    with open(os.path.join(H.ROOT, "tests", "golden", "ref_checksums.csv")) as f:
        return {(r["algo"], int(r["NP"]), int(r["SIZE"])): int(r["RESULT"]) for r in csv.DictReader(f, delimiter=";")}


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [4, 8] + H.wide(6))
def test_driver_golden_checksums(algo, p):
    """The drop-in drivers on the GPU against the reference's own recorded results
    (data/data_compare rows committed in tests/golden/ref_checksums.csv): every rank's
    printed checksum equals the reference's RESULT for that NP and SIZE -- the one-shot
    mesh (small sizes), the two-launch mesh (4 MiB) and, at NP = 6, the pre-step path."""
    gold = _golden_checksums()
    for size in (1, 64, 16384, 1 << 20):
        want = gold[(algo, p, size)]
        cp, hello = H.run_driver(algo, p, size, backend="gpu", env_extra={"FTAR_DEVMAP": ALL_ON_GPU0})
        assert cp.returncode == 0, (size, cp.stderr[-2000:])
        assert sorted(hello) == list(range(p)), (size, cp.stdout[-1000:])
        assert set(hello.values()) == {want}, (size, hello, want)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [12, 16])
def test_driver_golden_checksums_np_grid(algo, p):
    """The reference's own NP grid on the GPU (run/run_test.sh draws N in [4, 32]; its
    data_compare rows go up to NP = 64): the drop-in drivers at NP = 12 (Raben with 4 pre-step
    pairs, RD's reduce_pow2 over 4 extra ranks) and NP = 16 (the 16-source mesh tree, RD over
    4 steps) -- 12 / 16 rank processes time-sliced on one GPU, each with its own HIP context
    and 4 x (NP - 1) IPC imports -- every rank's checksum equal to the reference's RESULT at
    1, 16384 and 2^20 ints.  NP = 16 is the box's cap on processes that
    use the GPU at once; the host-sim covers NP up to 64 (tests/test_hostsim.py)."""
    gold = _golden_checksums()
    for size in (1, 16384, 1 << 20):
        want = gold[(algo, p, size)]
        cp, hello = H.run_driver(algo, p, size, backend="gpu", env_extra={"FTAR_DEVMAP": ALL_ON_GPU0}, timeout=240)
        assert cp.returncode == 0, (size, cp.stderr[-2000:])
        assert sorted(hello) == list(range(p)), (size, cp.stdout[-1000:])
        assert set(hello.values()) == {want}, (size, hello, want)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [4, 8])
def test_driver_golden_checksums_max_size(algo, p):
    """The reference's largest recorded size: 2^27 int32 (512 MiB) per rank
    (data/data_compare/{raben,rd}.csv, e.g. raben.csv:29 `4;134217728;...;805306368`),
    host buffers through the drop-in drivers, every rank's checksum equal to the
    reference's RESULT."""
    size = 1 << 27
    want = _golden_checksums()[(algo, p, size)]
    cp, hello = H.run_driver(algo, p, size, backend="gpu", env_extra={"FTAR_DEVMAP": ALL_ON_GPU0}, timeout=600)
    assert cp.returncode == 0, cp.stderr[-2000:]
    assert sorted(hello) == list(range(p)), cp.stdout[-1000:]
    assert set(hello.values()) == {want}, (hello, want)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("algo,p", [("raben", 3)] + H.wide(("rd", 2), ("raben", 2)))
def test_beyond_2g_elements(algo, p):
    """2^31 + 7 float32 elements per rank (8 GiB vectors, ~50 GiB of HBM per rank with the
    workspace): the C ABI takes size_t counts (the reference's int count stops at 2^31-1).
    bin/ftbench's pattern inputs x_r[i] = (7 i + 13 r) mod 4096 give every element its own
    exact sum, checked element by element on the host: window offsets and 64-bit indexing
    through the one-shot mesh (p = 2), recursive doubling and the pre-step path (p = 3)."""
    import json
    import subprocess
    n = (1 << 31) + 7
    env = dict(os.environ, FTBENCH_PATTERN="1")
    env.pop("FTAR_KILL", None)
    cp = subprocess.run([os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0,
                         os.path.join(H.PKG, "bin", "ftbench"), algo, str(n), "1"], env=env, capture_output=True,
                        text=True, timeout=800)
    assert cp.returncode == 0, cp.stderr[-2000:]
    lines = [json.loads(ln) for ln in cp.stdout.splitlines() if ln.startswith("{")]
    assert sorted(ln["rank"] for ln in lines) == list(range(p)), cp.stdout[-1000:]
    for ln in lines:
        c = ln["calls"][0]
        assert c["rc"] == 0 and c["comm_size"] == p and c["uniform"], ln


RELAY_ALL = {"FTAR_RELAY_MIN": "0", "FTAR_MESH": "0", "FTAR_RELAY": "1"}  # the step-by-step schedule, relayed


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [4, 6, 8, 9])
def test_relay_nofault(oracle, algo, p):
    """Exchanges striped over 2-hop relays (forced on for every window size)."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    o, r = _check(fn, algo, oracle.random_inputs(p, 100003, seed=p + 20), env=RELAY_ALL)
    assert min(st[0][8] for st in r.status.values()) > 0


@pytest.mark.parametrize("algo,kill", [("raben", (5, 1, 1, 1)), ("raben", (3, 1, 2, 1)), ("raben", (4, 2, 1, 1)),
                                       ("raben", (6, 1, 1, 2)), ("rd", (2, 1, 1, 1)), ("rd", (5, 1, 0, 1))])
def test_relay_kill(oracle, algo, kill):
    """A rank killed right after its relay phase: lost stripes are re-pulled directly."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    p = 9 if algo == "raben" else 8
    _check(fn, algo, oracle.random_inputs(p, 65536 + 7, seed=30), [kill], env=RELAY_ALL)


@pytest.mark.parametrize("algo,p,relay", [("raben", 8, True), ("rd", 8, True), ("raben", 9, False),
                                          ("rd", 5, False)])
def test_large_windows_interleaved(oracle, algo, p, relay):
    """Windows of many 64 KiB chunks: multi-segment launches take the interleaved block
    mapping (relay phases: up to 14 vector pieces from 7 peers; direct Raben step 0: the
    reduce half and the copy half)."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    o, r = _check(fn, algo, oracle.random_inputs(p, (1 << 22) + 13, seed=p + 40),
                  env=RELAY_ALL if relay else {"FTAR_RELAY": "0"})
    if relay:
        assert min(st[0][8] for st in r.status.values()) > 0


CE = {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0", "FTAR_MESH": "0"}


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [2, 5, 8])
def test_copy_engine_nofault(oracle, algo, p):
    """Direct pulls by hipMemcpyAsync (copy engine) + local reduce kernels."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    _check(fn, algo, oracle.random_inputs(p, 100003, seed=p + 50), env=CE)


@pytest.mark.parametrize("algo,kill", [("raben", (5, 1, 1, 2)), ("rd", (3, 1, 1, 2))])
def test_copy_engine_kill(oracle, algo, kill):
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    p = 9 if algo == "raben" else 8
    _check(fn, algo, oracle.random_inputs(p, 65536 + 9, seed=60), [kill], env=CE)


@pytest.mark.parametrize("p,kill", [(8, None), (4, None), (8, (3, 1, 1, 2)), (8, (5, 2, 1, 2))])
def test_raben_redundancy_always(oracle, p, kill):
    """The reference's step-0 full exchange kept at power-of-two p (FTAR_REDUNDANCY=1)."""
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(p, 100003, seed=p + 70),
           [kill] if kill else [], env={"FTAR_REDUNDANCY": "1"})


@pytest.mark.parametrize("algo,p,mode", [("raben", 4, "plain"), ("raben", 8, "inplace_offset3"), ("raben", 3, "inplace"),
                                         ("rd", 4, "offset1"), ("raben", 4, "inplace_mesh")] +
                         H.wide(("raben", 4, "inplace"), ("raben", 2, "offset1"), ("rd", 4, "inplace")))
def test_torch_device_buffers(oracle, algo, p, mode):
    """The device-pointer entry points on torch tensors (bench.py's path), bound through
    the Python package: in place, at element offsets, two calls; sbuf untouched.
    inplace_mesh: the two-launch mesh in place on device memory past the one-shot range (2 MiB),
    where the tree also stores this rank's final block into rbuf -- here sbuf -- while the
    peers read their blocks of it."""
    env = {"plain": {}, "inplace": {"FTAR_PROBE_INPLACE": "1"}, "offset1": {"FTAR_PROBE_OFFSET": "1"},
           "inplace_offset3": {"FTAR_PROBE_INPLACE": "1", "FTAR_PROBE_OFFSET": "3"},
           "inplace_mesh": dict(H.MESH_FORM, FTAR_PROBE_INPLACE="1", FTAR_ONESHOT_MAX="0")}[mode]
    env = dict(env, FTAR_STAGE_MAX="0")  # peers read sbuf in place (the path above 1 MiB)
    count = (1 << 19) + 64 if mode == "inplace_mesh" else 65536 + 17
    ins = oracle.random_inputs(p, count, seed=p + 90)
    o = (oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling)(ins)
    r = H.run_torch_worker(algo, ins, devmap=ALL_ON_GPU0, env_extra=env)
    assert r.returncode == 0, r.stderr[-2000:]
    for w in range(p):
        assert len(r.outputs.get(w, [])) == 2, r.stderr[-2000:]
        for it in range(2):
            assert r.status[w][it] == (0, 1), (w, it, r.status[w][it])
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("p", [4, 8])
def test_mesh_peer_wait(oracle, p):
    """The mesh's allgather ordered behind the peers' trees on the device (FTAR_OPT_MESH_WAIT,
    the default): one peer wait per call, none given up, one agree round fewer than the
    allgather after a host agree (FTAR_MESH_WAIT=0), bit-identical results (MAX over NaN /
    signed zeros pins every combination's operand order), two calls."""
    ins = H.with_specials(oracle.random_inputs(p, (1 << 20) + 3, seed=p + 170), p)
    o = oracle.rabenseifner(ins, op=2)
    runs = {}
    for wait in ("1", "0"):
        r = H.run_probe("raben", ins, op=2, iters=2, backend="gpu", devmap=ALL_ON_GPU0, timeout=300,
                        env_extra=dict(H.MESH_FORM, FTAR_ONESHOT_MAX="0", FTAR_MESH_WAIT=wait))
        assert r.returncode == 0, r.stderr[-2000:]
        for w in range(p):
            for it in range(2):
                assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (wait, w, it)
                assert r.status[w][it][15] == (1 if wait == "1" else 0) and r.status[w][it][16] == 0, r.status[w]
        runs[wait] = r
    assert all(runs["1"].status[w][0][7] == runs["0"].status[w][0][7] - 1 for w in range(p))


def test_mesh_peer_wait_timeout_fallback(oracle):
    """A rank publishes its flag 300 ms late (test hook, the hooks build): its peers' wait
    kernels give up after FTAR_GATE_TIMEOUT_MS and their allgathers return untouched; the
    verdicts travel in the last agree round, those ranks launch the allgather again -- exact
    results, the late rank's own wait not given up."""
    p, late = 4, 2
    ins = oracle.random_inputs(p, (1 << 20) + 3, seed=175)
    o = oracle.rabenseifner(ins)
    r = H.run_probe("raben", ins, iters=2, backend="gpu_hooks", devmap=ALL_ON_GPU0, timeout=300,
                    env_extra=dict(H.MESH_FORM, FTAR_ONESHOT_MAX="0", FTAR_GATE_TIMEOUT_MS="30",
                                   FTAR_PROBE_RANK_ENV=f"{late}:FTAR_PEER_WAIT_DELAY_US=300000"))
    assert r.returncode == 0, r.stderr[-2000:]
    for w in range(p):
        for it in range(2):
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)
            assert r.status[w][it][16] == (0 if w == late else 1), (w, it, r.status[w][it])


@pytest.mark.parametrize("kill", [(2, 1, 0, 0), (1, 1, 1, 3), (0, 2, 1, 3), (3, 2, 0, 1)])
def test_mesh_peer_wait_kills_abort(oracle, kill):
    """Kills around the device wait (p = 4, no idle rank: every failure aborts): before the
    tree -- the victim never publishes, the peers' wait kernels are given up by their failure
    detectors through the abort word --, with the tree in flight, during and after the
    allgather: a clean abort each time, never a hang."""
    ins = oracle.random_inputs(4, (1 << 20) + 3, seed=180 + kill[0])
    assert oracle.rabenseifner(ins, [kill]).aborted
    r = H.run_probe("raben", ins, [kill], backend="gpu", devmap=ALL_ON_GPU0, timeout=120,
                    env_extra=dict(H.MESH_FORM, FTAR_ONESHOT_MAX="0"))
    assert r.aborted and not r.outputs, r.stderr[-2000:]


MESH_SHAPES = [(2, 0, 100003), (4, 0, 100003), (8, 0, 65536 + 5), (4, 2, 4099), (8, 3, 4099), (4, 0, (1 << 22) + 13),
               (8, 1, (1 << 20) + 3)]
MESH_FORMS = [("0", "1"), ("1", "1"), ("2", "1"), ("0", "2"), ("0", "4"), ("1", "4")]
# every shape in the pull form, each other form on two shapes (a ragged / NaN-order one and a
# multi-workgroup one); the whole matrix under FTAR_GPU_WIDE=1
MESH_CASES = [s + f for f in MESH_FORMS for s in MESH_SHAPES] if H.WIDE else \
    [s + ("0", "1") for s in MESH_SHAPES] + \
    [s + f for f in MESH_FORMS[1:3] for s in (MESH_SHAPES[2], MESH_SHAPES[3])] + \
    [s + f for f in MESH_FORMS[3:] for s in (MESH_SHAPES[4], MESH_SHAPES[5])]


@pytest.mark.parametrize("p,op,count,push,unroll", MESH_CASES)
def test_mesh_schedule(oracle, p, op, count, push, unroll):
    """Power of two without a spare: one-hop reduce-scatter -- a tree kernel over p - 1
    peer pulls, or (FTAR_PUSH=1) p - 1 remote-store copies into the owners followed by the
    owner's tree over local memory -- and allgather (FTAR_PUSH=2: the owner's tree also
    stores its block into every peer), bit-identical to the step-by-step schedule; MAX/MIN
    with NaN and signed zeros pin the operand order of every combination.  FTAR_TREE_UNROLL
    = 2 / 4 (vectors per lane and source, p = 4, 8): the same tree per element, same bits --
    ragged lengths exercise the partial last workgroup and the scalar tail."""
    dt = np.int32 if op == 1 else np.float32
    ins = oracle.random_inputs(p, count, seed=p * 7 + op, dtype=dt)
    if op >= 2:
        ins = H.with_specials(ins, p + op)
    # one device-resident call (the host pipeline would split >= 16 MiB into chunk calls)
    o, r = _check(oracle.rabenseifner, "raben", ins, op=op,
                  env=dict(H.MESH_FORM, FTAR_ONESHOT_MAX="0", FTAR_HOST_PIPE="0", FTAR_PUSH=push,
                           FTAR_TREE_UNROLL=unroll))
    assert all(st[0][9] == 2 for st in r.status.values()), r.status


@pytest.mark.parametrize("p,op,count", [(2, 0, 100003), (4, 0, 4099), (8, 0, 65536 + 5), (4, 2, 4099), (8, 3, 4099),
                                        (8, 1, 7)])
def test_oneshot_schedule(oracle, p, op, count):
    """Small vectors at power of two without a spare: one launch evaluates every block in
    its owner's tree straight into rbuf, bit-identical to the step-by-step schedule --
    MAX/MIN with NaN and signed zeros pin the operand order."""
    dt = np.int32 if op == 1 else np.float32
    ins = oracle.random_inputs(p, count, seed=p * 11 + op, dtype=dt)
    if op >= 2:
        ins = H.with_specials(ins, p + op)
    o, r = _check(oracle.rabenseifner, "raben", ins, op=op, iters=2, env=dict(H.MESH_FORM, FTAR_ONESHOT_MAX=str(1 << 20)))
    u = np.uint32
    for w, st in r.status.items():
        assert st[0][9] == 1 and st[1][9] == 1, (w, st)
        assert np.array_equal(r.outputs[w][1].view(u), o.outputs[w].view(u)), w


@pytest.mark.parametrize("p,count,mode", [(8, 65536 + 5, {"FTAR_PROBE_INPLACE": "1"}),
                                          (8, (1 << 18) - 1, {"FTAR_PROBE_OFFSET": "1", "FTAR_PROBE_INPLACE": "1"}),
                                          (4, 1000, {"FTAR_PROBE_REALLOC": "1"})] +
                         H.wide((4, 4099, {}), (8, 7, {"FTAR_PROBE_OFFSET": "3"})))
def test_oneshot_device_buffers(oracle, p, count, mode):
    """The one-shot mesh on torch device buffers: peers read sbuf in place (staged when
    sbuf == rbuf), misaligned offsets, a re-allocated sbuf; sbuf never written."""
    ins = oracle.random_inputs(p, count, seed=p + count)
    o = oracle.rabenseifner(ins)
    r = H.run_torch_worker("raben", ins, devmap=ALL_ON_GPU0,
                           env_extra=dict(mode, FTAR_ONESHOT_MAX=str(1 << 20), FTAR_STAGE_MAX="0"))
    assert r.returncode == 0, r.stderr[-2000:]
    sign = -1 if mode.get("FTAR_PROBE_REALLOC") else 1
    for w in range(p):
        assert r.status[w][0] == (0, 1) and r.status[w][1] == (0, 1), r.status[w]
        assert np.array_equal(r.outputs[w][0].view(np.uint32), o.outputs[w].view(np.uint32))
        assert np.array_equal(r.outputs[w][1].view(np.uint32), (sign * o.outputs[w]).view(np.uint32))


MESH_KILLS = [(3, 1, 1, 2), (0, 2, 0, 1), (5, 1, 0, 0), (2, 1, 1, 3)]


# every kill in both pull forms, the push forms at two of them (all under FTAR_GPU_WIDE=1)
@pytest.mark.parametrize("kill,form", [(k, f) for f in ("0", str(1 << 20)) for k in MESH_KILLS] +
                         [(k, f) for f in ("push", "push2") for k in (MESH_KILLS if H.WIDE else MESH_KILLS[2:])])
def test_mesh_kill_aborts(oracle, kill, form):
    """Any death in the mesh phases (two-launch, one-shot, push) ends the job like the
    reference at p = 8 (no idle rank); (2, 1, 1, 3) dies mid-exchange with its peers'
    kernels reading (or, push, writing) its HBM."""
    env = {"FTAR_ONESHOT_MAX": "0", "FTAR_PUSH": "2" if form == "push2" else "1"} if form.startswith("push") \
        else {"FTAR_ONESHOT_MAX": form}
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(8, 10007, seed=kill[0]), [kill], env=env)


@pytest.mark.parametrize("p", [4, 8])
def test_mesh_staged_sbuf(oracle, p):
    """The mesh with sbuf staged in IN (FTAR_EXPORT=0) instead of read in place."""
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(p, 100003, seed=p + 600), env={"FTAR_EXPORT": "0"})


@pytest.mark.parametrize("algo,p", [("raben", 4), ("rd", 2)])
def test_full_size_256MiB(oracle, algo, p):
    """BASELINE's vector size (64 Mi float32 = 256 MiB per rank), bit-exact against the
    oracle: the mesh / step schedules with full-size windows (capped grids, pieces)."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    _check(fn, algo, oracle.random_inputs(p, 1 << 26, seed=p + 700))


@pytest.mark.parametrize("p", [4, 8])
def test_mesh_sbuf_reallocated(oracle, p):
    """A freed and re-allocated send buffer (likely the same address, a new allocation)
    is re-mapped by the peers: the second call (inputs negated) is exact."""
    ins = oracle.random_inputs(p, 1 << 20, seed=p + 800)
    o = oracle.rabenseifner(ins)
    r = H.run_torch_worker("raben", ins, devmap=ALL_ON_GPU0, env_extra={"FTAR_PROBE_REALLOC": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    for w in range(p):
        assert r.status[w][0] == (0, 1) and r.status[w][1] == (0, 1), r.status[w]
        assert np.array_equal(r.outputs[w][0].view(np.uint32), o.outputs[w].view(np.uint32))
        assert np.array_equal(r.outputs[w][1].view(np.uint32), (-o.outputs[w]).view(np.uint32))


@pytest.mark.parametrize("p,k,slices,inplace", [(4, 9, 0, 0), (2, 5, 0, 0), (4, 6, 1, 0), (4, 10, 0, 1)])
def test_send_buffer_cycling(tmp_path, p, k, slices, inplace):
    """A caller cycling its send buffer through more allocations than the peers' mapping
    cache holds (FTAR_UCACHE = 8; a bucketed all-reduce): every result exact, no mapping
    closed and re-opened per call (round 6 found such churn refused with 'invalid device
    pointer' at 4 ranks, and 8x slower calls at 2), the buffers beyond the cache staged.  slices:
    the buffers are views of one allocation at unaligned offsets (one entry, k offsets);
    inplace: every call with the send buffer as its receive buffer."""
    import subprocess
    import sys
    env = dict(os.environ, FTAR_PROBE_DIR=str(tmp_path), FTAR_CYCLE_BUFFERS=str(k), FTAR_CYCLE_SLICES=str(slices),
               FTAR_CYCLE_INPLACE=str(inplace))
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0, sys.executable, "-u",
           os.path.join(H.ROOT, "tests", "cycle_worker.py")]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert cp.returncode == 0, cp.stderr[-3000:]
    assert "mapping rank" not in cp.stderr and "not in this rank's cache" not in cp.stderr, cp.stderr[-3000:]
    for r in range(p):
        got = (tmp_path / f"cycle_{r}.txt").read_text()
        assert got.startswith("ok "), (r, got, cp.stderr[-2000:])
        # one 16 MiB call: far below the ~0.4 ms a mapping's close costs per peer
        assert float(got.split("median_us=")[1]) < 400, got


@pytest.mark.parametrize("p,kill", [(4, "2:1:1:3:6"), (5, "4:1:0:0:10")])
def test_send_buffer_cycling_through_a_kill(tmp_path, p, kill):
    """Recursive doubling with its callers cycling 9 send buffers, a rank killed in call 6 / 10
    (mid-exchange; at p = 5 the rank outside the power of two, before its step): the survivors
    recover and go on cycling on the shrunk comm -- the dead rank's mappings dropped, the
    survivors' mirrored caches in agreement -- every result uniform, calls before the kill
    summing every rank and calls after it the survivors'."""
    import json
    import subprocess
    import sys
    victim, call = int(kill.split(":")[0]), int(kill.split(":")[-1])
    env = dict(os.environ, FTAR_KILL=kill, FTAR_PROBE_DIR=str(tmp_path))
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0, sys.executable, "-u",
           os.path.join(H.ROOT, "tests", "kill_cycle_worker.py")]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [json.loads((tmp_path / f"kc_{r}.json").read_text()) for r in range(p) if (tmp_path / f"kc_{r}.json").exists()]
    assert sorted(ln["rank"] for ln in lines) == [r for r in range(p) if r != victim], (cp.returncode, cp.stderr[-3000:])
    assert "not in this rank's cache" not in cp.stderr and "mapping rank" not in cp.stderr, cp.stderr[-3000:]
    for ln in lines:
        for c, rec in enumerate(ln["calls"]):
            i = rec["buffer"]
            every = float(sum(r + 1 + 100 * i for r in range(p)))
            survivors = float(sum(r + 1 + 100 * i for r in range(p) if r != victim))
            assert rec["rc"] == 0 and rec["uniform"], (ln["rank"], c, rec)
            if c < call:
                assert rec["value"] == every and rec["size"] == p, (ln["rank"], c, rec)
            elif c == call:  # the victim's input counted or not, as the oracle's rules decide
                assert rec["value"] in (every, survivors) and rec["size"] == p - 1, (ln["rank"], c, rec)
            else:
                assert rec["value"] == survivors and rec["size"] == p - 1, (ln["rank"], c, rec)


@pytest.mark.parametrize("p,seed", [(4, 1), (3, 2), (8, 3)] + H.wide((4, 11), (5, 12), (2, 13), (6, 14)))
def test_random_call_sequences(tmp_path, p, seed):
    """120 calls drawn at random and alike on every rank -- schedule, dtype, every op the
    dtype allows, ragged lengths up to 3 Mi, element offsets, in place or not, fresh or
    re-used send buffers -- each result exact against the value every rank computes from all
    ranks' inputs (small integers: one exact answer in every dtype)."""
    import subprocess
    import sys
    env = dict(os.environ, FTAR_PROBE_DIR=str(tmp_path), FTAR_FUZZ_SEED=str(seed))
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0, sys.executable, "-u",
           os.path.join(H.ROOT, "tests", "fuzz_worker.py")]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert cp.returncode == 0, cp.stderr[-3000:]
    for r in range(p):
        assert (tmp_path / f"fuzz_{r}.txt").read_text() == "ok 120", (r, (tmp_path / f"fuzz_{r}.txt").read_text())


@pytest.mark.parametrize("seed", [1, 2, 3] + H.wide(4, 5, 6, 7, 8, 9))
def test_external_kill_while_cycling(tmp_path, seed):
    """A rank SIGKILLed from outside at a random instant of a 3000-call recursive-doubling
    loop (4 ranks cycling 9 device send buffers): the job either recovers -- every survivor's
    every result uniform, the full sum before the death, the survivors' sum after the comm
    shrank -- or ends in a clean MPI_Abort (the reference's rules abort a death in RD's first
    step); it never hangs and never returns a wrong value."""
    import random
    import signal
    import subprocess
    import sys
    import time
    rng = random.Random(seed)
    p = 4
    env = dict(os.environ, FTAR_PROBE_DIR=str(tmp_path))
    env.pop("FTAR_KILL", None)
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0, sys.executable, "-u",
           os.path.join(H.ROOT, "tests", "ext_kill_worker.py")]
    job = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        t0 = time.time()
        while not all((tmp_path / f"ready_{r}").exists() for r in range(p)):
            assert time.time() - t0 < 120 and job.poll() is None, "the job did not start"
            time.sleep(0.02)
        time.sleep(rng.uniform(0.0, 0.4))
        victim = rng.randrange(p)
        pids = subprocess.run(["pgrep", "-P", str(job.pid)], capture_output=True, text=True).stdout.split()
        ranks = {}
        for pid in pids:
            with open(f"/proc/{pid}/environ", "rb") as f:
                kv = dict(x.split(b"=", 1) for x in f.read().split(b"\0") if b"=" in x)
            ranks[int(kv[b"FTAR_RANK"])] = int(pid)
        os.kill(ranks[victim], signal.SIGKILL)
        out, err = job.communicate(timeout=180)
    finally:
        if job.poll() is None:
            job.kill()
    aborted = "MPI_ABORT" in err
    every = lambda i: float(sum(r + 1 + 100 * i for r in range(p)))
    surv = lambda i: float(sum(r + 1 + 100 * i for r in range(p) if r != victim))
    for r in range(p):
        if r == victim:
            continue
        lines = (tmp_path / f"xk_{r}.txt").read_text().split()
        recs = [lines[j:j + 6] for j in range(0, len(lines) - len(lines) % 6, 6)]
        shrunk = False
        for c, i, rc, size, v, uni in recs:
            i, rc, size, v = int(i), int(rc), int(size), float(v)
            assert rc == 0 and uni == "1", (r, c, rc, uni, err[-1500:])
            if size < p:
                assert v in (every(i), surv(i)) if not shrunk else v == surv(i), (r, c, v)
                shrunk = True
            else:
                assert v == every(i), (r, c, v)
        if not aborted:
            assert len(recs) == 3000 and shrunk, (r, len(recs), err[-1500:])
    assert aborted or job.returncode == 0, err[-2000:]
    import re
    code = re.search(r"errorcode (\d+)", err)
    # an abort is one the reference has: RD's check_abort (16), a fatal region (75)
    assert not aborted or (code and code.group(1) in ("16", "75")), err[-2000:]
    why = re.findall(r"ftar: rank \d+: [^\n]*", err)[:1]
    print(f"external kill of rank {victim}: " + (f"aborted (errorcode {code.group(1) if code else '?'}; {why})" if aborted
                                                 else "recovered"))


def test_peer_input_map_refused_falls_back():
    """The runtime refuses a peer send-buffer mapping (the hooks build's FTAR_FAIL_IMPORT: the
    13th import of every rank -- after the 4 x 3 workspace mappings -- gets a zeroed handle):
    every rank stages its input from then on, and the call and the next ones are exact.  The
    refusal leaves the runtime's sticky error behind; before round 6 it resurfaced as the
    fallback's next launch error and aborted the job."""
    import json
    import subprocess
    env = dict(os.environ, FTAR_FAIL_IMPORT="13")
    env.pop("FTAR_KILL", None)
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", "4", "--devmap", ALL_ON_GPU0,
           os.path.join(H.PKG, "bin", "ftbench_hooks"), "raben", str(1 << 22), "3"]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert cp.returncode == 0, cp.stderr[-3000:]
    assert "inputs are staged from now on" in cp.stderr, cp.stderr[-2000:]
    lines = [json.loads(x) for x in cp.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 4, cp.stdout[-2000:]
    for ln in lines:
        for call in ln["calls"]:
            assert call["rc"] == 0 and call["value"] == 6.0 and call["uniform"], ln


@pytest.mark.parametrize("p", [4, 3, 8])
def test_mixed_buckets_one_job(tmp_path, p):
    """A training step's gradient all-reduce as the library sees it: buckets of 7 .. 6 Mi
    elements in four dtypes, both schedules interleaved, some in place, each bucket its own
    buffer, four steps (forward and reversed order): every result exact."""
    import subprocess
    import sys
    env = dict(os.environ, FTAR_PROBE_DIR=str(tmp_path))
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0, sys.executable, "-u",
           os.path.join(H.ROOT, "tests", "bucket_worker.py")]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert cp.returncode == 0, cp.stderr[-3000:]
    for r in range(p):
        assert (tmp_path / f"bucket_{r}.txt").read_text() == "ok", (r, cp.stderr[-2000:])


@pytest.mark.parametrize("p,count", [(8, (1 << 23) + 77), (2, (1 << 22) + 5)])
def test_host_pipeline_chunks(oracle, p, count):
    """Host-buffer entry point at >= 16 MiB, power of two: chunk Allreduces with H2D and
    D2H on their own streams overlapping the exchanges, bit-exact to one call."""
    _check(oracle.rabenseifner, "raben", oracle.random_inputs(p, count, seed=p + 900))


@pytest.mark.parametrize("op", [2, 3])
def test_host_pipeline_operand_order(oracle, op):
    """Float MAX/MIN host calls >= 16 MiB stay one call (a chunk pipeline would move block
    owners and with them the operand order): NaN and signed zeros bit-exact."""
    p = 4
    ins = oracle.random_inputs(p, (1 << 22) + 77, seed=p + 40 * op)
    rng = np.random.default_rng(p + op)
    for x in ins:
        k = rng.integers(0, x.size, 1 << 16)
        x[k[: 1 << 15]] = np.nan
        x[k[1 << 15:]] = rng.choice(np.array([0.0, -0.0], dtype=np.float32), 1 << 15)
    _check(oracle.rabenseifner, "raben", ins, op=op)


@pytest.mark.parametrize("p", [4, 8])
def test_growing_sizes_one_job(tmp_path, p):
    """Sizes 4 KiB .. 256 MiB in one job with fresh send buffers at every size: the
    workspace grows and is re-exported while peers hold mappings of earlier buffers."""
    import subprocess
    import sys
    env = dict(os.environ, FTAR_PROBE_DIR=str(tmp_path))
    cmd = [os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ALL_ON_GPU0, sys.executable, "-u",
           os.path.join(H.ROOT, "tests", "grow_worker.py")]
    cp = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert cp.returncode == 0, cp.stderr[-3000:]
    for r in range(p):
        # right results, and no IPC export refused (nor re-allocated) at any growth
        assert (tmp_path / f"grow_{r}.txt").read_text() == "ok retries=0", (r, cp.stderr[-2000:])


@pytest.mark.parametrize("algo", ["raben", "rd"])
def test_device_entry_refuses_pageable_host_memory(algo):
    """Pageable host memory handed to the device entry points: FTAR_ERR_ARG on every rank
    before anything is launched (no device fault), and the comm stays usable."""
    rng = np.random.default_rng(5)
    ins = [rng.standard_normal(1031).astype(np.float32) for _ in range(2)]
    r = H.run_probe(algo, ins, iters=2, backend="gpu", devmap=ALL_ON_GPU0, timeout=120,
                    env_extra={"FTAR_PROBE_DEVICE": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    for w in range(2):
        assert r.status[w][0][0] == 13 and r.status[w][1][0] == 13, r.status[w]


@pytest.mark.parametrize("algo,p,env", [
    ("raben", 8, {"FTAR_ONESHOT_MAX": "0"}), ("raben", 9, {"FTAR_RELAY_MIN": "0"}), ("rd", 6, {"FTAR_RELAY_MIN": "0"}),
    ("rd", 8, {}), ("raben", 9, {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0"})] +
    H.wide(("raben", 4, {}), ("raben", 2, {})))
def test_capped_grids_plain_stores(oracle, algo, p, env):
    """One workgroup per CU (FTAR_BLOCKS_PER_CU=1: 256-workgroup grids) so every kernel
    strides over its pieces and the tree launches split, with plain instead of
    non-temporal stores (FTAR_NT_STORE=0): the launch geometry and store flavour change,
    the bits must not -- MAX over NaN / signed zeros pins every operand order."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    ins = H.with_specials(oracle.random_inputs(p, (1 << 20) + 37, seed=p * 13 + 5), p + 1)
    _check(fn, algo, ins, op=2, env=dict(env, FTAR_BLOCKS_PER_CU="1", FTAR_NT_STORE="0"))
    _check(fn, algo, oracle.random_inputs(p, (1 << 20) + 37, seed=p * 13 + 6),
           env=dict(env, FTAR_BLOCKS_PER_CU="1"))


def _bit_inputs(p, n, seed, dt):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(p):
        v = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        v[rng.random(n) < 0.3] = 0
        out.append(v)
    return out


@pytest.mark.parametrize("algo,p,op,count,env", [
    ("raben", 8, 9, 100003, {"FTAR_ONESHOT_MAX": "0", "FTAR_HOST_PIPE": "0"}),   # mesh (tree kernel)
    ("raben", 8, 4, 4099, {}),                                                   # one-shot (tree batch)
    ("raben", 4, 7, 65541, {"FTAR_MESH": "0"}),                                  # step by step
    ("raben", 5, 6, 65541, {}),                                                  # pre/post-step + relay
    ("raben", 2, 5, 100003, {}),
    ("rd", 8, 8, 65541, {}),
    ("rd", 6, 9, 4099, {"FTAR_RELAY": "0"}),
    ("raben", 4, 9, 65541, {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0", "FTAR_MESH": "0"})])
def test_schedule_logical_bitwise(oracle, algo, p, op, count, env):
    """MPI's logical / bitwise ops (int32 / int64) through every kernel form the schedules
    use -- tree, tree batch, segment, copy engine + local reduce -- bit-exact to the oracle."""
    dt = np.int64 if op % 2 else np.int32
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    _check(fn, algo, _bit_inputs(p, count, p * 17 + op, dt), op=op, env=env)


@pytest.mark.parametrize("algo,p,kill,op", [("raben", 9, (6, 1, 1, 3), 9), ("raben", 9, (6, 2, 1, 3), 4),
                                            ("rd", 6, (3, 1, 1, 3), 7)])
def test_kill_logical_bitwise(oracle, algo, p, kill, op):
    """A kill mid-exchange under a bitwise op: recovery replays with the call's op."""
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    o, _ = _check(fn, algo, _bit_inputs(p, 65541, p + op, np.int32), [kill], op=op)
    assert not o.aborted and o.recoveries >= 1


@pytest.mark.parametrize("algo,p,mode", [("raben", 2, {}), ("raben", 8, {"FTAR_PROBE_INPLACE": "1", "FTAR_ONESHOT_MAX": "0"}),
                                         ("raben", 5, {}), ("raben", 4, {"FTAR_MESH": "0", "FTAR_PROBE_OFFSET": "1"}),
                                         ("rd", 6, {"FTAR_PROBE_INPLACE": "1"})] +
                         H.wide(("raben", 4, {}), ("raben", 4, {"FTAR_ONESHOT_MAX": "0"}), ("rd", 4, {})))
def test_pinned_host_buffers(oracle, algo, p, mode):
    """The device entry points on pinned host buffers: this rank's kernels read sbuf and
    write rbuf in place over PCIe (zero copy), peers read the staged copy in HBM (host
    memory is never exported).  One-shot, mesh, spare, step-by-step and RD forms; in
    place and at element offsets; two calls; sbuf untouched; bit-exact to the oracle."""
    ins = oracle.random_inputs(p, 65536 + 17, seed=p + 190)
    o = (oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling)(ins)
    r = H.run_torch_worker(algo, ins, devmap=ALL_ON_GPU0, env_extra=dict(mode, FTAR_PROBE_PINNED="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    for w in range(p):
        assert len(r.outputs.get(w, [])) == 2, r.stderr[-2000:]
        for it in range(2):
            assert r.status[w][it] == (0, 1), (w, it, r.status[w][it])
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("algo,p,kills,env", [
    ("rd", 4, [], {}), ("rd", 6, [(3, 1, 1, 3)], {}), ("rd", 8, [(5, 1, 1, 2)], {"FTAR_PROBE_OFFSET": "1"}),
    ("raben", 5, [], {}), ("raben", 9, [(6, 1, 1, 3)], {}), ("raben", 5, [(3, 2, 0, 1)], {"FTAR_PROBE_INPLACE": "1"}),
    ("raben", 4, [], {"FTAR_HOST_PIPE": "0"}), ("raben", 4, [], {})])
def test_host_entry_pinned_zero_copy(oracle, algo, p, kills, env):
    """The _host entry points on pinned caller buffers (hipHostMalloc): where the call is
    not chunk-pipelined they run the device entry point on the caller's buffers in place
    (zero copy over PCIe, no staging), including kills mid-exchange and recoveries;
    bit-exact to the oracle, sbuf untouched."""
    ins = oracle.random_inputs(p, 65536 + 9, seed=p * 13 + len(kills))
    _check(oracle.recursive_doubling if algo == "rd" else oracle.rabenseifner, algo, ins, kills,
           env=dict(env, FTAR_PROBE_PINNED="1"))


# The stated float tolerance (north_star "within a stated tolerance for float
# SUM"): bit-exact against the oracle's tree (the tests above), and against the exact sum
# |err_i| <= gamma(depth) * sum_r |x_r[i]| per element, gamma(d) = d u / (1 - d u), u = 2^-24
# (the standard bound of a summation tree of height d in round-to-nearest), depth = the
# reduction tree's height (ceil(log2 p): the pre-step of a non-power-of-two p adds one level).
FLOAT_TOL_UNIT = 2.0 ** -24


@pytest.mark.timeout(300)
@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [2, 5, 8])
def test_float_sum_within_stated_tolerance(oracle, algo, p):
    """float32 SUM of uniform [-1, 1) vectors (1 Mi + 3 elements per rank) against the exact
    sum in float64: every element within gamma(depth) x sum |x|, on every rank."""
    ins = oracle.random_inputs(p, (1 << 20) + 3, seed=300 + p)
    r = H.run_probe(algo, ins, backend="gpu", devmap=ALL_ON_GPU0, timeout=240)
    assert r.returncode == 0 and not r.aborted, r.stderr[-2000:]
    exact = np.sum([x.astype(np.float64) for x in ins], axis=0)
    mag = np.sum([np.abs(x.astype(np.float64)) for x in ins], axis=0)
    depth = int(np.ceil(np.log2(p)))
    bound = depth * FLOAT_TOL_UNIT / (1 - depth * FLOAT_TOL_UNIT) * mag
    for w in range(p):
        err = np.abs(r.outputs[w][0].astype(np.float64) - exact)
        assert (err <= bound).all(), (w, float((err / np.maximum(bound, 1e-300)).max()))


@pytest.mark.parametrize("name,value", [("FTAR_FLAG_MAX_BLOCKS", "lots"), ("FTAR_TREE_UNROLL", "3"),
                                        ("FTAR_NT_STORE", "off"), ("FTAR_GATE_TIMEOUT_MS", "0")])
def test_device_knob_refused(oracle, name, value):
    """A device-layer knob that is not a whole number in its range is refused when the rank
    opens its device (the job fails with one line naming it), never read as 0 the way atoi
    would read it."""
    ins = oracle.random_inputs(2, 1031, seed=5)
    r = H.run_probe("raben", ins, backend="gpu", devmap=ALL_ON_GPU0, timeout=120, env_extra={name: value})
    assert r.returncode != 0 and not r.outputs
    assert f"{name}={value} is not " in r.stderr and "refused" in r.stderr, r.stderr[-1500:]
