"""The product's host C under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md 5:
the reference has no sanitizer runs; its own code writes through a const sbuf).

tests/hostsim is rebuilt into _build_asan with -fsanitize=address,undefined
-fno-sanitize-recover=all: control plane, both schedules, both error handlers, the
transport (relay stripes, copy engine), the launcher and the probe.  Any sanitizer
report aborts the rank with a nonzero status, which fails the comparison below.  Ranks
that die by injected SIGKILL or leave through MPI_Abort's _exit skip the leak check;
every clean exit runs it.
"""
import fcntl
import os
import subprocess

import numpy as np
import pytest

import harness as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ("-O1 -g -std=c11 -Wall -Wno-unused-parameter -fPIC -D_GNU_SOURCE -fsanitize=address,undefined "
         "-fno-sanitize-recover=all -fno-omit-frame-pointer")


@pytest.fixture(scope="module")
def asan_build():
    # one build at a time (pytest-xdist workers share the output directory)
    with open(os.path.join(ROOT, "tests", "hostsim", ".asan.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "hostsim"), "OUT=_build_asan",
                        f"CFLAGS={FLAGS}", "all"], check=True)
    return H.HOSTSIM_ASAN


def _run(oracle, algo, ins, kills=(), env=None, iters=1):
    fn = oracle.rabenseifner if algo == "raben" else oracle.recursive_doubling
    o = fn(ins, kills)
    e = dict(ASAN_OPTIONS="abort_on_error=1:detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1", **(env or {}))
    r = H.run_probe(algo, ins, kills, iters=iters, backend="hostsim_asan", timeout=300, env_extra=e)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-3000:]
    assert "LeakSanitizer" not in r.stderr, r.stderr[-3000:]
    if o.aborted:
        assert r.aborted, r.stderr[-2000:]
        return
    assert not r.aborted and r.returncode == 0, r.stderr[-3000:]
    for w, st in enumerate(o.status):
        if st == 0:
            for it in range(iters):
                assert np.array_equal(r.outputs[w][it].view(np.uint32), o.outputs[w].view(np.uint32)), (w, it)


@pytest.mark.parametrize("algo", ["raben", "rd"])
@pytest.mark.parametrize("p", [1, 2, 3, 5, 8, 9])
def test_asan_nofault(asan_build, oracle, algo, p):
    _run(oracle, algo, oracle.random_inputs(p, 1031, seed=p + 200), iters=2)


@pytest.mark.parametrize("algo,p,env", [("raben", 8, {"FTAR_RELAY_MIN": "0", "FTAR_MESH": "0"}), ("raben", 8, {}),
                                        ("rd", 6, {"FTAR_RELAY_MIN": "0"}),
                                        ("raben", 9, {"FTAR_COPY_ENGINE": "1", "FTAR_RELAY": "0"}),
                                        ("raben", 4, {"FTAR_PROBE_DEVICE": "1", "FTAR_PROBE_INPLACE": "1",
                                                      "FTAR_PROBE_OFFSET": "3"})])
def test_asan_transports(asan_build, oracle, algo, p, env):
    _run(oracle, algo, oracle.random_inputs(p, 3001, seed=p + 300), env=env)


@pytest.mark.parametrize("algo,p,kill", [("raben", 9, (5, 1, 1, 2)), ("raben", 9, (4, 2, 1, 1)),
                                         ("raben", 11, (3, 1, 2, 0)), ("rd", 8, (3, 1, 1, 2)),
                                         ("rd", 6, (1, 1, 1, 2)), ("raben", 8, (2, 1, 1, 2)),
                                         ("raben", 9, (5, 1, 1, 3)), ("raben", 11, (2, 1, 2, 3)),
                                         ("rd", 8, (3, 1, 1, 3))])
def test_asan_recovery(asan_build, oracle, algo, p, kill):
    """Error handlers (impersonation replay, state hand-off, regroup; RD spare and shrink
    branches) and the abort path, relayed where the windows allow it.  Point 3 kills the
    victim mid-exchange (pre-image restore on the partner, late correction)."""
    _run(oracle, algo, oracle.random_inputs(p, 2053, seed=p + 400), [kill], env={"FTAR_RELAY_MIN": "0"})


@pytest.mark.parametrize("algo,p", [("raben", 4), ("rd", 5)])
def test_asan_send_buffer_caches(asan_build, oracle, algo, p):
    """The mirrored send-buffer caches (ftar_comm.c xcache_admit / peer_sbuf) under the
    sanitizers: 12 exportable send buffers cycled, so entries are admitted, hit and (beyond
    the eighth) staged on exporter and importers alike."""
    seq = list(range(8)) + [8, 9] * 7 + list(range(12)) + [3, 2, 1, 0]
    env = {"FTAR_PROBE_DEVICE": "1", "FTAR_PROBE_CYCLE_SEQ": ",".join(map(str, seq)), "FTAR_STAGE_MAX": "0"}
    _run(oracle, algo, oracle.random_inputs(p, 3001, seed=p + 500), env=env, iters=len(seq))
