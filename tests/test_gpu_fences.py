"""Cross-device fence discipline on the GPU.

Every rank of a device-resident job (bin/ftbench under ftrun, all ranks on GPU 0) logs its
launches, drains, fenced markers, gate verdicts and barriers (FTAR_TRACE), and
tests/fence_check.py checks the two rules the node's cross-GPU visibility rests on over
all ranks' logs: every peer read after barrier k sees only writes their owner released at
system scope before arriving at k, and the reading launch invalidates (acquire) or follows
a fenced marker with no stale read of that range in between.  On one GPU a violation cannot
give a wrong result (one HBM behind the same L2s), so the discipline is checked directly,
for every transport form and across the small-call thresholds.  A deliberately removed
release (FTAR_TRACE_DROP=release: the marker drains without their system fence) and a
removed acquire (FTAR_TRACE_DROP=acquire) must each fail it.

FTAR_GPU_FENCE_WIDE=1 adds the 8-rank and remaining size/form combinations."""
import json
import os
import shutil
import subprocess
import tempfile

import pytest

import fence_check as FC
import harness as H

pytestmark = pytest.mark.gpu

MIB = 1 << 20
# (ranks, algo, float32 elements, options): every form and the sizes on both sides of the
# small-call thresholds (1 MiB: staging, one-shot, gates, completion flags)
BASE = [
    (2, "raben", 1, {}),                                   # 4 B: one-shot, staged, gated
    (4, "raben", 16384, {}),                               # 64 KiB one-shot
    (4, "raben", 262140, {}),                              # 1 MiB - 16 B
    (4, "raben", 262148, {}),                              # 1 MiB + 16 B: two-launch mesh, read in place
    (4, "raben", MIB, {}),                                 # 4 MiB mesh (allgather behind a device wait)
    (4, "raben", MIB, {"FTAR_MESH_WAIT": "0"}),            # 4 MiB mesh, allgather after a host agree
    (16, "raben", MIB, {}),                                # 16-source tree, 15 flags per wait
    (4, "raben", MIB, {"FTAR_TREE_UNROLL": "2"}),          # mesh_u2
    (8, "raben", MIB, {"FTAR_TREE_UNROLL": "4"}),          # mesh_u4, 8 ranks
    (4, "raben", MIB, {"FTAR_PUSH": "1"}),                 # mesh_push
    (4, "raben", MIB, {"FTAR_PUSH": "2"}),                 # mesh_push2
    (4, "raben", 16384, {"FTAR_PUSH": "2", "FTAR_ONESHOT_MAX": "0"}),
    (4, "raben", MIB, {"FTAR_GATE_MAX": str(16 * MIB), "FTAR_MESH_WAIT": "0"}),  # mid-size gate: allgather behind the tree
    (4, "raben", MIB, {"FTAR_MESH": "0", "FTAR_RELAY": "1", "FTAR_RELAY_MIN": "0"}),  # relay2hop
    (4, "raben", MIB, {"FTAR_MESH": "0", "FTAR_RELAY": "0"}),                         # direct
    (4, "raben", MIB, {"FTAR_MESH": "0", "FTAR_COPY_ENGINE": "1"}),                   # copy engine
    (5, "raben", MIB, {}),                                 # spare: pre-step, step by step, post-step
    (3, "raben", 16384, {}),
    (4, "rd", 1, {}),
    (4, "rd", 16384, {}),                                  # gated steps, staged
    (4, "rd", 262148, {}),
    (4, "rd", MIB, {"FTAR_GATE_MAX": str(16 * MIB)}),      # mid-size gated steps 1..
    (4, "rd", MIB, {"FTAR_RELAY_MIN": "0"}),               # relayed steps
    (5, "rd", 16384, {}),                                  # pre-step + fan-out
    (4, "raben", 16384, {"FTAR_FLAG_SYNC": "0"}),          # fenced-marker drains only
    # kills mid-exchange (configs[4]'s shape at 5 ranks = 4 + idle spare): the recovery's
    # launches -- the impersonator's replay of the dead rank's steps, the corr reduce, the new
    # entry's state pulls -- read the dead rank's and the survivors' memory across barriers too
    (5, "raben", MIB, {"FTAR_KILL": "3:1:1:3:1"}),         # RS step 1, DURING, call 1
    (5, "raben", MIB, {"FTAR_KILL": "4:2:0:3:1"}),         # last AG step, DURING
    (5, "rd", 16384, {"FTAR_KILL": "1:1:1:3:1"}),          # RD step 1, DURING
    (4, "raben", 64 * MIB, {}),                            # 256 MiB mesh
    (4, "raben", 64 * MIB, {"FTAR_MESH_WAIT": "0"}),       # the headline size, allgather after a host agree
]
WIDE = [
    (8, "raben", 1, {}), (8, "raben", 16384, {}), (8, "raben", 262140, {}), (8, "raben", 262148, {}),
    (8, "raben", MIB, {}), (8, "raben", MIB, {"FTAR_PUSH": "2"}),
    (8, "raben", MIB, {"FTAR_MESH": "0", "FTAR_RELAY_MIN": "0"}), (8, "rd", MIB, {"FTAR_RELAY_MIN": "0"}),
    (8, "rd", 16384, {}), (2, "rd", 262148, {}), (2, "raben", 64 * MIB, {}), (8, "raben", 64 * MIB, {}),
]
CASES = BASE + (WIDE if os.environ.get("FTAR_GPU_FENCE_WIDE") == "1" else [])


def _trace_job(p, algo, n, opts, drop=None, calls=3):
    tmp = tempfile.mkdtemp(prefix="ftar_fence_")
    # pattern inputs (every element its own exact sum) without kills; rank ids with one
    env = {k: v for k, v in os.environ.items() if k not in ("FTAR_KILL", "FTAR_TRACE_DROP")}
    env.update(opts, FTBENCH_PATTERN="0" if "FTAR_KILL" in opts else "1", FTAR_TRACE=os.path.join(tmp, "t"))
    if drop:  # the drop hook lives only in the TEST-ONLY hooks build of the library
        env["FTAR_TRACE_DROP"] = drop
    bench = "ftbench_hooks" if drop else "ftbench"
    cp = subprocess.run([os.path.join(H.PKG, "bin", "ftrun"), "-np", str(p), "--devmap", ",".join("0" * p),
                         os.path.join(H.PKG, "bin", bench), algo, str(n), str(calls)], env=env,
                        capture_output=True, text=True, timeout=240)
    lines = [json.loads(ln) for ln in cp.stdout.splitlines() if ln.startswith("{")]
    logs = FC.load(os.path.join(tmp, "t"))
    shutil.rmtree(tmp, ignore_errors=True)
    assert sorted(logs) == list(range(p))
    if "FTAR_KILL" not in opts:
        assert cp.returncode == 0, cp.stderr[-2000:]
        assert sorted(ln["rank"] for ln in lines) == list(range(p)), cp.stdout[-1000:]
        for ln in lines:
            assert all(c["rc"] == 0 and c["uniform"] for c in ln["calls"]), ln
        return FC.check(logs), logs
    # a kill: the victim is gone, every survivor completed every call, all with the same
    # value per call (inputs are the rank ids), and the comm shrank by one; Raben's kill call
    # keeps the victim's contribution (the impersonator's replay), later calls are the
    # survivors' sum
    victim = int(opts["FTAR_KILL"].split(":")[0])
    assert "dies mid-exchange" in cp.stderr, cp.stderr[-2000:]
    assert sorted(ln["rank"] for ln in lines) == [r for r in range(p) if r != victim], cp.stdout[-1000:]
    full, rest = float(sum(range(p))), float(sum(range(p)) - victim)
    for ln in lines:
        cs = ln["calls"]
        assert all(c["rc"] == 0 and c["uniform"] for c in cs), ln
        assert [c["value"] for c in cs] == [c["value"] for c in lines[0]["calls"]], (ln, lines[0])
        assert cs[0]["value"] == full and cs[-1]["value"] == rest, ln
        if algo == "raben":
            assert cs[1]["value"] == full, ln
        assert cs[1]["recoveries"] == 1 and cs[-1]["comm_size"] == p - 1, ln
    rep = FC.check(logs)
    if algo == "raben" and opts["FTAR_KILL"].split(":")[1] == "1":
        # the reduce-scatter replay read the dead rank's step-0 input where it lies (one GPU:
        # the copy is elided), and that read was checked against the dead rank's releases
        assert rep.dead_reads > 0
    return rep, logs


@pytest.mark.timeout(300)
@pytest.mark.parametrize("p,algo,n,opts", CASES, ids=[f"{a}-p{p}-{4 * n}B-" + ("_".join(f"{k[5:]}{v}" for k, v in o.items())
                                                                                 or "default")
                                                      for p, a, n, o in CASES])
def test_fence_discipline(p, algo, n, opts):
    rep, logs = _trace_job(p, algo, n, opts)
    assert rep.ok, (rep.release[:5], rep.acquire[:5])
    assert rep.reads_checked > 0  # peer reads were seen and checked
    assert all(lg.arrive and lg.passed for lg in logs.values())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("wait", ["1", "0"])
def test_dropped_release_fails_the_check(wait):
    """The mesh's tree is released by a fenced marker -- in front of the flag the peers'
    allgathers wait for on the device (FTAR_MESH_WAIT=1), or drained before the reduce-scatter's
    barrier (0); with that marker's system fence removed (test-only switch) the allgather's
    peer reads of the blocks it wrote are unreleased reads, and the checker says so."""
    rep, _ = _trace_job(4, "raben", MIB, {"FTAR_MESH_WAIT": wait}, drop="release")
    assert rep.release, "a removed release went unnoticed"
    if wait == "1":
        assert any("before flag" in v for v in rep.release), rep.release[:3]


@pytest.mark.timeout(300)
def test_dropped_acquire_fails_the_check():
    """Small RD calls drain by completion flags only; each gated step invalidates its caches
    before reading the peers' accumulators.  With the acquires removed the next call's reads
    of lines the previous call cached are stale reads, and the checker says so."""
    rep, _ = _trace_job(4, "rd", 16384, {}, drop="acquire")
    assert rep.acquire, "a removed acquire went unnoticed"
