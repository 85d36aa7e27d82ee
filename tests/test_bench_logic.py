"""bench.py's host-side logic on CPU: the configs[4] leg's launch line and its summary
(which call is the kill call, the exact-sum checks before and after the shrink, the
medians), driven by a stand-in for ftrun + ftbench that prints what the real ranks print.
The leg itself runs on the node in the driver's scaling run (and on one GPU in
tests/test_gpu_bench.py)."""
import importlib.util
import json
import os
import stat

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FAKE_FTRUN = r'''#!/usr/bin/env python3
# stand-in for ftrun -np N --devmap ... ftbench raben COUNT CALLS: one JSON line per
# surviving rank, as bin/ftbench prints them
import json, os, sys
a = sys.argv[1:]
n = int(a[a.index("-np") + 1])
devmap = a[a.index("--devmap") + 1]
calls = int(a[-1])
kill = os.environ.get("FTAR_KILL")
with open(os.environ["FAKE_LOG"], "a") as f:
    f.write(json.dumps({"argv": a, "kill": kill}) + "\n")
victim, kc = (int(kill.split(":")[0]), int(kill.split(":")[4])) if kill else (-1, -1)
full = float(sum(range(n)))
for r in range(n):
    if r == victim:
        continue
    cs = []
    for c in range(calls):
        after = kill and c > kc
        cs.append({"rc": 0, "ms": 2.0 + (1.5 if c == kc else 0) + (5 if c == 0 else 0) - (0.5 if after else 0),
                   "recoveries": 1 if c == kc else 0, "comm_size": n - 1 if kill and c >= kc else n,
                   "value": full - victim if after else full, "uniform": True})
    print(json.dumps({"rank": r, "size": n, "device": 0, "calls": cs}))
if kill:
    sys.stderr.write(f"ftar: rank {victim} dies mid-exchange (phase 1 step 1): own kernel in flight, {n - 1} peers launched\n")
'''


@pytest.fixture
def bench(tmp_path, monkeypatch):
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    bindir = tmp_path / "fault-tolerant_amd" / "bin"
    bindir.mkdir(parents=True)
    f = bindir / "ftrun"
    f.write_text(FAKE_FTRUN)
    f.chmod(f.stat().st_mode | stat.S_IEXEC)
    (bindir / "ftbench").write_text("")
    monkeypatch.setattr(m, "ROOT", str(tmp_path))
    monkeypatch.setattr(m, "c5_random_kill", lambda *a, **k: {"stub": True})
    monkeypatch.setenv("FAKE_LOG", str(tmp_path / "log.jsonl"))
    return m, tmp_path


def test_c5_leg_summary(bench):
    m, tmp = bench
    res = m.c5_leg(8, list(range(8)), 1024, 9)
    assert res["devmap"] == [0, 0, 1, 2, 3, 4, 5, 6, 7]  # ranks 0, 1 (pre-step pair + idle spare) on GPU 0
    assert res["recovered"] is True, res
    assert res["kill"].startswith("6:1:1:3 in call 2")
    f, n = res["fault"], res["no_fault"]
    assert f["survivors"] == 8 and n["survivors"] == 9
    assert all(c["result_ok"] for c in f["calls"]) and all(c["result_ok"] for c in n["calls"])
    assert [c["comm_size_after"] for c in f["calls"]] == [9, 9, 8, 8, 8, 8]
    assert res["recovered_call_ms"] == 3.5 and res["no_fault_call_ms"] == 2.0
    assert res["pre_fault_call_ms"] == 2.0 and res["survivors_call_ms"] == 1.5
    assert res["recovery_overhead_ms"] == 1.5
    assert "dies mid-exchange" in f["victim"]
    assert res["recovered_rs"] and res["recovered_ag"] and res["recovered_ag_call_ms"] == 3.5
    assert res["kill_ag"].startswith("6:2:1:3 in call 2")
    runs = [json.loads(l) for l in open(tmp / "log.jsonl")]
    assert [r["kill"] for r in runs] == [None, "6:1:1:3:2", "6:2:1:3:2"]
    assert runs[0]["argv"][-3:] == ["raben", "1024", "6"]


def test_c5_leg_rehearsal_layout(bench):
    """One GPU, 5 ranks (FTAR_C5_RANKS): the victim is the last rank."""
    m, _ = bench
    res = m.c5_leg(2, [0], 64, 5)
    assert res["devmap"] == [0, 0, 0, 0, 0] and res["kill"].startswith("4:1:1:3 in call 2")
    assert res["kill_ag"].startswith("4:2:0:3 in call 2")  # two AG steps: the last one recovers
    assert res["recovered"] is True, res


def test_c5_leg_wrong_sum_is_not_recovered(bench, monkeypatch):
    """A survivor whose result misses the exact sum fails the leg."""
    m, tmp = bench
    f = tmp / "fault-tolerant_amd" / "bin" / "ftrun"
    f.write_text(FAKE_FTRUN.replace('"value": full - victim if after else full', '"value": full'))
    res = m.c5_leg(8, list(range(8)), 1024, 9)
    assert res["recovered"] is False
    assert not all(c["result_ok"] for c in res["fault"]["calls"])


def test_side_legs_run_on_rank0_before_torch(bench, monkeypatch):
    """The side legs (CPU baseline, configs[4] jobs, fabric probe) run on rank 0 only, and
    rank 0 writes the flag the other ranks wait on even when a leg raises; the other
    ranks return as soon as the flag exists.  Neither imports torch (the ranks are not
    GPU processes while the legs run: tools/kfd_probe.py)."""
    import argparse
    import sys
    m, tmp = bench
    monkeypatch.setenv("MASTER_PORT", f"t{os.getpid()}")
    calls = []

    def c5(world, devices, count, ranks):
        calls.append((world, devices, count, ranks))
        raise RuntimeError("leg failed")

    monkeypatch.setattr(m, "c5_leg", c5)
    monkeypatch.setattr(m, "cpu_schedule", lambda *a: (_ for _ in ()).throw(OSError("no cores")))
    monkeypatch.setenv("FTAR_C5_RANKS", "9")
    args = argparse.Namespace(count=1 << 10, no_cpu_baseline=False, no_c5=False, no_xgmi=True)
    had_torch = "torch" in sys.modules
    flag = m.leg_flag("side")
    assert not os.path.exists(flag)
    try:
        cpu, c5r, xg = m.side_legs(args, 0, 8, list(range(8)), False)
        assert os.path.exists(flag)
        assert calls == [(8, list(range(8)), 1 << 10, 9)]
        assert c5r == {"error": "leg failed"} and xg is None
        assert cpu["value"] is None and "no cores" in cpu["sample"] and cpu["cores"] == 8
        assert m.side_legs(args, 3, 8, list(range(8)), False) == (None, None, None)
        assert len(calls) == 1
        if not had_torch:
            assert "torch" not in sys.modules
    finally:
        if os.path.exists(flag):
            os.unlink(flag)
