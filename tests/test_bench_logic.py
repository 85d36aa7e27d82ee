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
    f.write(json.dumps({"argv": a, "kill": kill, "redundancy": os.environ.get("FTAR_REDUNDANCY")}) + "\n")
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


def _deadline(s=60.0):
    import time
    return time.monotonic() + s


def test_c5_leg_summary(bench):
    m, tmp = bench
    res = m.c5_leg(8, list(range(8)), 1024, 9, _deadline())
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
    # both recovery shapes: the library's default (auto: the ranks span GPUs, so the
    # reference's step-0 copy moves), then the opt-in elided shape (FTAR_REDUNDANCY=0)
    assert [r["kill"] for r in runs] == [None, "6:1:1:3:2", "6:2:1:3:2"] * 2
    assert [r["redundancy"] for r in runs] == [None] * 3 + ["0"] * 3
    assert runs[0]["argv"][-3:] == ["raben", "1024", "6"]
    assert "span GPUs" in res["recovery_shape"] and "reference_shape" not in res
    el = res["elided_shape"]
    assert el["recovered"] and el["recovered_rs"] and el["recovered_ag"], el
    assert el["no_fault"]["survivors"] == 9 and el["fault"]["survivors"] == 8
    assert res["dead_input_cross_device"] == el["dead_input_cross_device"] == "recovered"


def test_c5_leg_elided_shape_abort_is_reported(bench):
    """On the node the elided shape's RS-kill job decides whether a dead process's memory
    stays readable across GPUs: an MPI_Abort there reads `dead_input_cross_device: abort`
    (the default shape, with the copy, still recovers)."""
    m, tmp = bench
    f = tmp / "fault-tolerant_amd" / "bin" / "ftrun"
    f.write_text(FAKE_FTRUN.replace("if kill:\n    sys.stderr.write(",
                                    "if kill and os.environ.get('FTAR_REDUNDANCY') == '0' and kill.split(':')[1] == '1':\n"
                                    "    sys.stderr.write('MPI_ABORT was invoked on rank 1\\n'); sys.exit(1)\n"
                                    "if kill:\n    sys.stderr.write(")
                 .replace("for r in range(n):\n    if r == victim:",
                          "for r in range(n):\n    if kill and os.environ.get('FTAR_REDUNDANCY') == '0' and "
                          "kill.split(':')[1] == '1':\n        break\n    if r == victim:"))
    res = m.c5_leg(8, list(range(8)), 1024, 9, _deadline())
    assert res["recovered"] is True, res
    assert res["dead_input_cross_device"] == "abort", res["elided_shape"]["fault"]


def test_c5_leg_rehearsal_layout(bench):
    """One GPU, 5 ranks (FTAR_C5_RANKS): the victim is the last rank; the default is the
    elided shape there, the other shape the reference's copy."""
    m, tmp = bench
    res = m.c5_leg(2, [0], 64, 5, _deadline())
    assert res["devmap"] == [0, 0, 0, 0, 0] and res["kill"].startswith("4:1:1:3 in call 2")
    assert res["kill_ag"].startswith("4:2:0:3 in call 2")  # two AG steps: the last one recovers
    assert res["recovered"] is True, res
    assert "one GPU" in res["recovery_shape"] and res["reference_shape"]["recovered"]
    assert "dead_input_cross_device" not in res
    runs = [json.loads(l) for l in open(tmp / "log.jsonl")]
    assert [r["redundancy"] for r in runs] == [None] * 3 + ["1"] * 3


def test_c5_leg_wrong_sum_is_not_recovered(bench, monkeypatch):
    """A survivor whose result misses the exact sum fails the leg."""
    m, tmp = bench
    f = tmp / "fault-tolerant_amd" / "bin" / "ftrun"
    f.write_text(FAKE_FTRUN.replace('"value": full - victim if after else full', '"value": full'))
    res = m.c5_leg(8, list(range(8)), 1024, 9, _deadline())
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

    def c5(world, devices, count, ranks, deadline):
        calls.append((world, devices, count, ranks))
        raise RuntimeError("leg failed")

    monkeypatch.setattr(m, "c5_leg", c5)
    monkeypatch.setattr(m, "c5_campaign", lambda *a, **k: {"stub": True})
    monkeypatch.setattr(m, "cpu_schedule", lambda *a, **k: (_ for _ in ()).throw(OSError("no cores")))
    monkeypatch.setenv("FTAR_C5_RANKS", "9")
    args = argparse.Namespace(count=1 << 10, no_cpu_baseline=False, no_c5=False, no_xgmi=True, side_budget=30.0,
                              c5_draws=2)
    had_torch = "torch" in sys.modules
    flag = m.leg_flag("side")
    assert not os.path.exists(flag)
    try:
        cpu, c5r, xg, info = m.side_legs(args, 0, 8, list(range(8)), False)
        assert os.path.exists(flag)
        assert calls == [(8, list(range(8)), 1 << 10, 9)]
        assert c5r == {"error": "leg failed", "random_kill_campaign": {"stub": True}} and xg is None
        assert cpu["value"] is None and "no cores" in cpu["sample"] and cpu["cores"] == 8
        assert info["c5"]["status"] == "error" and info["cpu_baseline"]["status"] == "error"
        assert m.side_legs(args, 3, 8, list(range(8)), False) == (None, None, None, None)
        assert len(calls) == 1
        if not had_torch:
            assert "torch" not in sys.modules
    finally:
        if os.path.exists(flag):
            os.unlink(flag)


def test_run_proc_kills_the_whole_group(bench):
    """A side-leg job past its deadline is killed with every process it forked (ftrun's
    ranks are in the launcher's process group)."""
    import time
    m, tmp = bench
    pidfile = tmp / "child.pid"
    t0 = time.monotonic()
    rc, out, err, to = m.run_proc(["bash", "-c", f"sleep 300 & echo $! > {pidfile}; wait"], 1.5)
    assert to and time.monotonic() - t0 < 10
    child = int(pidfile.read_text())
    time.sleep(0.2)
    assert not os.path.exists(f"/proc/{child}") or open(f"/proc/{child}/stat").read().split()[2] == "Z"


def test_side_leg_past_its_deadline_is_recorded(bench, monkeypatch):
    """FTAR_BENCH_HANG=c5: the configs[4] leg's stand-in job never ends; the side legs still
    end inside their one budget, the leg reads "timeout" and the campaign gets the rest."""
    import argparse
    import time
    m, tmp = bench
    monkeypatch.setenv("MASTER_PORT", f"h{os.getpid()}")
    monkeypatch.setenv("FTAR_BENCH_HANG", "c5")
    monkeypatch.setattr(m, "cpu_schedule", lambda *a, **k: ({"time_s": 0.1, "algbw_GBps": 1.0,
                                                              "cpu_s_per_rank_whole_process": 0.1}, "cpu"))
    seen = []
    monkeypatch.setattr(m, "c5_campaign", lambda dev, count, ranks, d, draws=10: seen.append(d - time.monotonic())
                        or {"draws_run": 0})
    args = argparse.Namespace(count=1 << 10, no_cpu_baseline=False, no_c5=False, no_xgmi=True, side_budget=8.0,
                              c5_draws=2)
    t0 = time.monotonic()
    try:
        cpu, c5r, xg, info = m.side_legs(args, 0, 8, list(range(8)), False)
    finally:
        flag = m.leg_flag("side")
        if os.path.exists(flag):
            os.unlink(flag)
    took = time.monotonic() - t0
    assert took < 8.0 + 3.0, took
    assert info["c5"]["status"] == "timeout" and "killed" in c5r["error"], (info, c5r)
    assert cpu["value"] and info["cpu_baseline"]["status"] == "ok"
    assert seen and 0 < seen[0] <= 8.0 * 0.65 + 0.5  # the campaign runs on what is left


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_ns", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _fracs(d):
    """Every value under a key named `frac` or ending in `_frac`, recursively."""
    out = []
    for k, v in d.items():
        if isinstance(v, dict):
            out += _fracs(v)
        elif k == "frac" or k.endswith("_frac"):
            out.append(v)
    return out


def test_north_star_block_prices():
    """FT Raben moves 2.25 S per rank and direction at p = 8 over one link per
    step; at B_link = 153.6 GB/s t_roof = 3.93 ms and the 70 % target is algbw >= 47.8 GB/s.
    The top-level fraction is the timed schedule against its OWN bound: the
    one-hop mesh moves 2 S / 8 over each link, 0.874 ms at 76.8 GB/s."""
    m = _bench_module()
    S = 256 << 20
    # a synthetic node line: mesh 1.3 ms, the reference's shape 9 ms, calibrated link 76.8 GB/s
    ns = m.north_star_block(8, S, 1.3e-3, "mesh", 76.8, 7, 2.0 * S / 8, t_ref=9e-3)
    assert ns["basis"] == "calibrated" and ns["applies"]
    t_sched = 2.0 * S / 8 / 76.8e9
    assert ns["frac"] == round(t_sched / 1.3e-3, 4) and ns["met"] is False  # 0.672 < 0.70
    t_roof = 2.25 * S / 76.8e9
    assert ns["reference_schedule_frac"] == round(t_roof / 9e-3, 4) and ns["reference_schedule_met"] is True
    assert ns["speedup_vs_survey_roofline"] == round(t_roof / 1.3e-3, 4) > 1  # a speed-up, not a fraction
    assert all(f is None or f <= 1.0 for f in _fracs(ns)), _fracs(ns)
    row = ns["priced"]["survey_153.6_assumed"]
    assert abs(row["survey_t_roof_ms"] - 3.9322) < 1e-3 and abs(row["survey_target_algbw_GBps"] - 47.78) < 0.05
    assert abs(ns["priced"]["nominal_76.8_assumed"]["survey_t_roof_ms"] - 7.8643) < 1e-3
    # met follows the schedule's own fraction
    fast = m.north_star_block(8, S, 1.2e-3, "mesh", 76.8, 7, 2.0 * S / 8)
    assert fast["met"] is True and fast["frac"] == round(t_sched / 1.2e-3, 4)
    # a time below its own bound (the reference's shape in 6 ms, faster than 2.25 S over one
    # 76.8 GB/s link allows): no fraction above 1 is claimed, the price is flagged instead
    bad = m.north_star_block(8, S, 1.3e-3, "mesh", 76.8, 7, 2.0 * S / 8, t_ref=6e-3)
    assert bad["reference_schedule_frac"] is None and bad["reference_schedule_met"] is None
    assert bad["priced"]["calibrated"]["reference_schedule"]["frac_raw"] > 1
    assert all(f is None or f <= 1.0 for f in _fracs(bad)), _fracs(bad)
    # no calibration: priced at SURVEY's 153.6 GB/s assumption (the strictest)
    nocal = m.north_star_block(8, S, 5.0e-3, "mesh", None, 7, 2.0 * S / 8)
    assert nocal["basis"] == "survey_153.6_assumed"
    assert nocal["frac"] == round(2.0 * S / 8 / 153.6e9 / 5.0e-3, 4)
    reh = m.north_star_block(2, S, 1e-3, "mesh-oneshot", None, 1, S, rehearsal=True)
    assert reh["frac"] is None and reh["met"] is None and reh["rehearsal"]


def test_rd_roofline_and_non_kernel_time():
    """configs[2] (RD, 256 MiB, 8 GPUs) gets a link roofline on the node
    line, and the headline's north-star block carries the call's time outside kernels.  A
    synthetic node line: RD relayed in 3.2 ms (its own bound: 3 steps x 2 S / 8 over each of
    7 links = 2.62 ms at 76.8 GB/s), the direct transport -- the reference's movement, L S
    over one link per step, 10.49 ms -- in 11.5 ms; the mesh headline 1.3 ms of which 1.0 ms
    kernels."""
    m = _bench_module()
    S = 256 << 20
    rd = m.rd_roofline_block(8, S, 3.2e-3, "relay2hop", 76.8, t_direct=11.5e-3,
                             breakdown={"call_ms": 3.3, "kernels_ms": 2.9})
    t_own = 3 * 2.0 * S / 8 / 76.8e9
    t_ref = 3.0 * S / 76.8e9
    assert rd["links"] == 7 and rd["schedule_bytes_per_link"] == 3 * 2.0 * S / 8
    assert rd["frac"] == round(t_own / 3.2e-3, 4) and rd["frac"] <= 1.0
    assert rd["reference_schedule_frac"] == round(t_ref / 11.5e-3, 4) <= 1.0
    assert rd["speedup_vs_reference_roofline"] == round(t_ref / 3.2e-3, 4) > 1  # a speed-up, not a fraction
    assert abs(rd["non_kernel_ms"] - 0.4) < 1e-9 and rd["kernels_ms"] == 2.9
    assert all(f is None or f <= 1.0 for f in _fracs(rd)), _fracs(rd)
    # direct: the reference's own data movement, one link per step
    d = m.rd_roofline_block(8, S, 11.5e-3, "direct", 76.8, t_direct=11.5e-3)
    assert d["links"] == 1 and d["frac"] == d["reference_schedule_frac"] == round(t_ref / 11.5e-3, 4)
    # p = 9 (a spare): the pre-step and the fan-out each move one more vector on the path
    d9 = m.rd_roofline_block(9, S, 20e-3, "direct", 76.8)
    assert d9["reference_bytes_per_rank"] == 5.0 * S
    # a time below the bound claims no fraction above 1
    fast = m.rd_roofline_block(8, S, 2.0e-3, "relay2hop", 76.8)
    assert fast["frac"] is None and "bound_violated" in fast
    # one-GPU rehearsal: printed, fractions withheld
    reh = m.rd_roofline_block(2, S, 1e-3, "direct", None, t_direct=1e-3, rehearsal=True)
    assert reh["frac"] is None and reh["reference_schedule_frac"] is None
    # the north-star block: time outside kernels beside the fraction
    ns = m.north_star_block(8, S, 1.3e-3, "mesh", 76.8, 7, 2.0 * S / 8,
                            breakdown={"call_ms": 1.3, "kernels_ms": 1.0, "agree_barrier_wait_ms": 0.2,
                                       "stream_drain_wait_ms": 0.1})
    assert abs(ns["non_kernel_ms"] - 0.3) < 1e-9 and ns["kernels_ms"] == 1.0
    assert ns["non_kernel_share"] == round(0.3 / 1.3, 4)
    assert ns["frac_kernels_only"] == round(2.0 * S / 8 / 76.8e9 / 1.0e-3, 4) <= 1.0
    assert all(f is None or f <= 1.0 for f in _fracs(ns)), _fracs(ns)


def _torchrun_cpu(tmp_path, extra_env, extra_args, timeout, nproc=2, count=65536):
    import socket
    import subprocess
    import sys
    import time
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, FTAR_BENCH_CPU_TEST="1", FTAR_HOSTSIM_TAG=f"bench{os.getpid()}", **extra_env)
    for k in ("FTAR_JOB", "FTAR_RANK", "FTAR_SIZE", "FTAR_LAUNCHER", "FTAR_KILL", "FTAR_DEVICE"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--device",
           "cpu", "--dist-backend", "gloo", "--count", str(count), "--steps", "3", "--warmup", "1"] + extra_args
    t0 = time.monotonic()
    cp = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    subprocess.run(f"rm -f /dev/shm/ftarhs-bench{os.getpid()}-*", shell=True)
    lines = [json.loads(l) for l in cp.stdout.splitlines() if l.startswith("{")]
    return cp, lines, time.monotonic() - t0


@pytest.mark.timeout(240)
def test_bench_multi_headline_survives_hung_and_failing_legs(hostsim, tmp_path):
    """The N > 1 line under the driver's launch line (torchrun, 2 ranks), on CPU with the
    host-sim library: the configs[4] side leg hangs past its deadline, one transport and the
    RD leg fail.  The headline line is printed right after configs[3] is timed, with the
    contract's keys and the north-star block; the final line completes with every leg's
    fate recorded, inside the budgets."""
    cp, lines, took = _torchrun_cpu(tmp_path, {"FTAR_BENCH_HANG": "c5", "FTAR_BENCH_FAIL": "transports:direct,rd"},
                                    ["--side-budget", "20", "--c5-draws", "1"], 200)
    assert cp.returncode == 0, cp.stderr[-3000:]
    assert [d["line"] for d in lines] == ["headline", "final"], cp.stdout[-2000:]
    head, fin = lines
    for d in lines:
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                  "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "north_star"):
            assert k in d, k
        assert d["value"] > 0 and d["n_gpus"] == 2 and "CPU TEST" in d["data"]
        ns = d["north_star"]
        assert ns["target"] and ns["priced"]["survey_153.6_assumed"]["survey_t_roof_ms"] > 0 and "met" in ns
    assert head["value"] == fin["value"]
    assert fin["side_legs"]["c5"]["status"] == "timeout" and "killed" in fin["c5_single_kill"]["error"]
    assert fin["side_legs"]["total_s"] <= 20 + 2
    assert fin["transports"]["direct"]["error"].startswith("transports:direct: forced failure")
    assert fin["transports"]["relay2hop"]["raben_ms"] > 0
    assert fin["legs"]["rd"]["status"] == "error" and fin["rd"] is None
    assert "non_kernel_ms" in fin["north_star"] and fin["north_star"]["kernels_ms"] >= 0
    assert fin["exact_on_node"]["all_exact"], fin["exact_on_node"]
    assert fin["int32_rank_checksum_ok"] == {"raben": True, "rd": True}
    assert fin["cpu_baseline"]["value"] and fin["cpu_baseline"]["cores"] == 2
    # what the run decides (analysis/analyze.py decisions), in the line itself
    nd = fin["node_decisions"]
    assert "error" not in nd, nd
    assert nd["n_gpus"] == 2 and nd["all_exact"] and nd["gate_max_bytes"] >= 1 << 20, nd
    # the sweep ends one point past the job's vector, as the reference's campaign (2^27 ints)
    sweep = fin["size_sweep_us"]
    assert sweep[str(8 * 65536)]["raben_us"] > 0 and sweep[str(8 * 65536)]["rd_us"] > 0, sweep
    assert took < 150, took


@pytest.mark.timeout(240)
def test_bench_multi_small_call_fallback(hostsim, tmp_path):
    """exact_on_node covers every small-call mechanism on both sides of its ~1 MiB threshold,
    gated and ungated.  With a gated path that is not exact
    (FTAR_HOSTSIM_GATE_CORRUPT: a gated launch's first output element is off by one), the
    gated checks fail, the leg reruns them with the gates off, finds them exact, keeps that
    setting for the rest of the job and records it; the size sweep is timed with it."""
    cp, lines, took = _torchrun_cpu(tmp_path, {"FTAR_HOSTSIM_GATE_CORRUPT": "1"},
                                    ["--side-budget", "5", "--no-c5", "--no-xgmi", "--no-cpu-baseline"], 200)
    assert cp.returncode == 0, cp.stderr[-3000:]
    fin = lines[-1]
    ex = fin["exact_on_node"]
    assert not ex["all_exact"], ex
    fb = ex["small_call_fallback"]
    assert fb["setting"] == "gate=0" and fb["tried"][0] == {"setting": "gate=0", "exact": True,
                                                             "still_inexact": []}, fb
    # the gated small checks, and every check of the job's own 256 KiB vector that is gated
    # too (RD at a power of two, the one-shot mesh forms) -- never an ungated one
    assert "rd_4B_gated" in fb["failed"] and not any(n.endswith("_ungated") for n in fb["failed"]), fb
    assert ex["all_exact_after_fallback"] is True, ex
    for label in ("4B", "4KiB", "64KiB", "1MiB-16B", "1MiB", "1MiB+16B"):  # --count 65536 = 256 KiB: 4 MiB skipped
        for algo in ("raben", "rd"):
            assert f"{algo}_{label}_ungated" in ex or 4 * {"4B": 1, "4KiB": 1024, "64KiB": 16384}.get(label, 1 << 30) \
                > 4 * 65536, (algo, label)
    assert ex["rd_4B_ungated"] and not ex["rd_4B_gated"]
    sweep = fin["size_sweep_us"]
    assert sweep["small_call_setting"] == "gate=0" and sweep["gate"] == 0, sweep
    assert fin["transport_selection"]["inexact"], fin["transport_selection"]  # the gated one-shot failed there too
    # configs[2]'s roofline block rides on the RD leg (fractions withheld off the node)
    rl = fin["rd"]["schedule_link_roofline"]
    assert rl["transport"] == "direct" and rl["links"] == 1 and rl["frac"] is None and rl["rehearsal"], rl
    assert rl["reference_bytes_per_rank"] == 4.0 * 65536 and "non_kernel_ms" in rl, rl


@pytest.mark.timeout(240)
def test_bench_multi_watchdog_prints_and_exits(hostsim, tmp_path):
    """An optional leg that never returns (FTAR_BENCH_HANG=checks): at the job budget the
    watchdog prints the line as it stands (marked truncated) and every rank exits cleanly."""
    cp, lines, took = _torchrun_cpu(tmp_path, {"FTAR_BENCH_HANG": "checks"},
                                    ["--side-budget", "5", "--budget", "30", "--no-c5", "--no-xgmi"], 200)
    assert cp.returncode == 0, cp.stderr[-3000:]
    assert [d["line"] for d in lines] == ["headline", "final"], cp.stdout[-2000:]
    assert "watchdog" in lines[-1]["truncated"] and lines[-1]["value"] == lines[0]["value"]
    assert took < 30 + 30, took


@pytest.mark.timeout(240)
def test_bench_multi_four_ranks_device_wait(hostsim, tmp_path):
    """Four ranks, 4 MiB per rank (above the one-shot and gate limits): the default mesh orders
    its allgather behind the peers' trees on the device (the transports leg counts its peer
    waits); the transport selection times `mesh_host_ag` -- the allgather after a host agree
    round -- beside the others, exact_on_node checks it at the job's size, node_decisions says
    whether the device wait was faster, and configs[2]'s roofline block carries L = 2 steps of
    the reference's movement."""
    cp, lines, took = _torchrun_cpu(tmp_path, {}, ["--side-budget", "5", "--no-c5", "--no-xgmi", "--no-cpu-baseline"],
                                    200, nproc=4, count=1 << 20)
    assert cp.returncode == 0, cp.stderr[-3000:]
    fin = lines[-1]
    sel = fin["transport_selection"]
    assert "mesh_ms" in sel and not sel["inexact"] and not sel["failed"], sel
    assert fin["exact_on_node"]["all_exact"], fin["exact_on_node"]
    assert fin["transports"]["mesh"]["peer_waits"] > 0, fin["transports"]["mesh"]
    nd = fin["node_decisions"]
    # the device-ordered allgather (default) against the host-agree form: timed, exact, decided
    assert "mesh_host_ag_ms" in sel and fin["exact_on_node"]["mesh_host_ag"], (sel, fin["exact_on_node"])
    assert nd["device_wait_faster"] in (True, False), nd
    assert "mesh_host_ag" in fin["transports"], fin["transports"]
    rl = fin["rd"]["schedule_link_roofline"]
    assert rl["reference_bytes_per_rank"] == 2.0 * 4 * (1 << 20), rl
    assert "non_kernel_ms" in fin["north_star"], fin["north_star"]


FAKE_ROCPROF = r'''#!/usr/bin/env python3
# stand-in for rocprofv3 --pmc CTR -d DIR -o pmc --output-format csv -- CHILD...: writes the
# counter CSV a real pass writes (one row per dispatch), values as gfx950 reports them
import os, sys
a = sys.argv[1:]
ctr, d = a[a.index("--pmc") + 1], a[a.index("-d") + 1]
child = a[a.index("--") + 1:]
assert child[1].endswith("bench.py") and "--pmc-child" in child, child
os.makedirs(os.path.join(d, "host"), exist_ok=True)
val = {"FETCH_SIZE": 131080.0, "WRITE_SIZE": 262144.0}[ctr]  # KiB: half-counted reads, exact writes
with open(os.path.join(d, "host", "77_counter_collection.csv"), "w") as f:
    f.write('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n')
    f.write(f'1,"void at::native::elementwise_kernel",{ctr},5.0\n')
    for i in range(20):
        f.write(f'{i + 2},"void ftar::reduce_lds_kernel<float, 0>(...)",{ctr},{val}\n')
'''


def test_pmc_live_passes_and_correction(tmp_path, monkeypatch):
    """The N = 1 line's `roofline.traffic` is measured in the run: two
    rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a `bench.py --pmc-child`, averaged over
    the C2 kernel's dispatches and corrected for gfx950 (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B).
    Here a stand-in rocprofv3 writes the CSVs; the real passes run in the bench on the box."""
    import argparse
    import shutil
    m = _bench_module()
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE_ROCPROF)
    fake.chmod(0o755)
    monkeypatch.setattr(shutil, "which", lambda n: str(fake) if n == "rocprofv3" else None)
    monkeypatch.delenv("LD_PRELOAD", raising=False)
    args = argparse.Namespace(count=1 << 26, pairs=4, variant=1, no_pmc=False)
    traffic, src = m.pmc_live(args, "reduce_lds_kernel")
    assert traffic == round((2 * 131080.0 + 262144.0) * 1024), src
    assert src["measured_in_this_run"] and src["dispatches"] == [20, 20], src
    assert all(p["rc"] == 0 for p in src["passes"].values()), src
    # skipped, and said why, under a profiler or with --no-pmc
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    assert m.pmc_live(args, "reduce_lds_kernel") == (None, {"measured_in_this_run": False,
                                                           "skipped": "already under a profiler"})
    monkeypatch.delenv("ROCPROF_OUTPUT_PATH")
    args.no_pmc = True
    assert m.pmc_live(args, "reduce_lds_kernel")[1]["skipped"] == "--no-pmc"
