"""GPU: launches queued behind gates when a peer is late (ADVICE r03, high + medium + low).

A gated launch (Raben's one-shot, every RD step at a power of two, <= 1 MiB) is queued
before the barrier that readies its operands and spins at the head of the rank's stream
until the host opens its gate.  A late peer must cost neither the job nor a bounded stall:
  * the host gives the gated launch up once its barrier waited FTAR_GATE_HOLD_US (the step
    then launches after the barrier) -- `gate_holds`;
  * with the host hold off, the device gives the gate up after FTAR_GATE_TIMEOUT_MS (its
    workgroups return without touching memory) and the next drain relaunches the plan
    ungated -- `gate_relaunches` -- instead of failing the call; for RD that drain is the one
    with step s + 1 already queued behind its own gate (the verify the gate-pending branch
    used to skip).
Every result bit-exact against the oracle.  All ranks on GPU 0 of the test box.
"""
import numpy as np
import pytest

import harness as H

pytestmark = pytest.mark.gpu

ALL_ON_GPU0 = ",".join(["0"] * 16)


def _run(oracle, algo, p, env, iters=3, count=1031):
    ins = oracle.random_inputs(p, count, seed=p + 17)
    o = oracle.rabenseifner(ins) if algo == "raben" else oracle.recursive_doubling(ins)
    # the last rank is late: small calls -- it arrives 300 ms late (its calls' first barrier
    # has the gated launch pending); mid-size calls -- it stretches its steps to 300 ms
    # (FTAR_LOOP_SECONDS: the barriers of steps 1.. / the reduce-scatter's agree, behind which
    # the next launch is gated)
    late = {"FTAR_PROBE_RANK_ENV": f"{p - 1}:FTAR_PROBE_SLEEP_US=300000" if count <= 4096 else
            f"{p - 1}:FTAR_LOOP_SECONDS=0.3", "FTAR_RELAY": "0", "FTAR_HOST_PIPE": "0", "FTAR_GATE_MAX": str(16 << 20),
            **H.MESH_FORM, **H.GATES_ON}
    r = H.run_probe(algo, ins, iters=iters, backend="gpu", devmap=ALL_ON_GPU0, timeout=120, env_extra=dict(late, **env))
    assert r.returncode == 0 and not r.aborted, r.stderr[-2000:]
    for w in range(p):
        for it in range(iters):
            assert r.status[w][it][0] == 0, r.status[w]
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)
    return r


@pytest.mark.timeout(180)
@pytest.mark.parametrize("algo,p,count", [("raben", 4, 1031), ("rd", 4, 1031), ("rd", 2, 1031),
                                          ("rd", 4, (1 << 19) + 3)])
def test_late_peer_host_gives_gate_up(oracle, algo, p, count):
    """(2 MiB: RD's mid-size relayed gates, whose barriers wait for the late rank's steps)"""
    r = _run(oracle, algo, p, {"FTAR_GATE_HOLD_US": "2000", "FTAR_ONESHOT_MAX": "0" if count > 4096 else str(1 << 20)},
             count=count)
    # call 0 allocates the workspace, whose collective absorbs the late arrival before any gate
    assert all(r.status[w][it][13] >= 1 for w in range(p - 1) for it in (1, 2)), r.status
    assert all(r.status[w][it][14] == 0 for w in range(p) for it in range(3)), r.status  # no device timeout


@pytest.mark.timeout(240)
@pytest.mark.parametrize("algo,p,count", [("rd", 4, (1 << 19) + 3), ("rd", 8, (1 << 21) + 5), ("rd", 2, (1 << 22) - 7)])
def test_mid_size_gates(oracle, algo, p, count):
    """Mid-size calls (2 MiB .. 16 MiB, FTAR_GATE_MAX = 16 MiB; off by default):
    RD's steps 1.. are queued ahead of their barriers behind gates relayed through device memory (one workgroup polls
    the host word), the grid capped at half the CUs so ranks sharing the GPU still run; the
    drain before the barrier waits on a fenced marker recorded in front of the gated launch.
    Bit-exact against the oracle (MAX over NaN / signed zeros for the operand order)."""
    ins = H.with_specials(oracle.random_inputs(p, count, seed=p + 23), p)
    o = oracle.rabenseifner(ins, op=2) if algo == "raben" else oracle.recursive_doubling(ins, op=2)
    r = H.run_probe(algo, ins, op=2, iters=3, backend="gpu", devmap=ALL_ON_GPU0, timeout=200,
                    env_extra={"FTAR_RELAY": "0", "FTAR_ONESHOT_MAX": "0", "FTAR_HOST_PIPE": "0", **H.MESH_FORM,
                               **H.GATES_ON, "FTAR_GATE_TIMEOUT_MS": "10000",
                               "FTAR_GATE_MAX": str(16 << 20)})
    assert r.returncode == 0 and not r.aborted, r.stderr[-2000:]
    per_call = p.bit_length() - 2
    for w in range(p):
        for it in range(3):
            st = r.status[w][it]
            assert st[0] == 0 and st[10] == per_call and st[14] == 0, (w, it, st)
            assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("algo,p,count", [("raben", 4, 1031), ("rd", 4, 1031), ("rd", 2, 1031),
                                          ("rd", 4, (1 << 19) + 3)])
def test_late_peer_device_gate_timeout_relaunches(oracle, algo, p, count):
    r = _run(oracle, algo, p, {"FTAR_GATE_HOLD_US": "0", "FTAR_GATE_TIMEOUT_MS": "30",
                               "FTAR_ONESHOT_MAX": "0" if count > 4096 else str(1 << 20)}, count=count)
    assert all(r.status[w][it][13] == 0 for w in range(p) for it in range(3)), r.status  # the host never gave up
    # the waiting ranks' gated launches timed out on the device and were relaunched
    assert all(r.status[w][2][14] >= 1 for w in range(p - 1)), r.status
    assert "relaunched" in r.stderr, r.stderr[-1500:]


@pytest.mark.timeout(180)
@pytest.mark.parametrize("algo,p,count", [("raben", 4, 1031), ("rd", 4, 1031), ("rd", 4, (1 << 19) + 3)])
def test_device_timeout_then_host_hold_never_relaunches(oracle, algo, p, count):
    """The device gives the gate up first (30 ms), then the host's hold (100 ms) gives the
    launch up as well and the step launches after the barrier: the kept plan must not run
    again at the next drain (it could be stale by then, e.g. after a recovery)."""
    r = _run(oracle, algo, p, {"FTAR_GATE_HOLD_US": "100000", "FTAR_GATE_TIMEOUT_MS": "30",
                               "FTAR_ONESHOT_MAX": "0" if count > 4096 else str(1 << 20)}, count=count)
    assert all(r.status[w][it][13] >= 1 for w in range(p - 1) for it in (1, 2)), r.status
    assert all(r.status[w][it][14] == 0 for w in range(p) for it in range(3)), r.status
    assert "relaunched" not in r.stderr, r.stderr[-1500:]
