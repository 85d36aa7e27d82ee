"""bench.py's two paths as the driver runs them, on the one-GPU test box.

N = 1: `python bench.py` -- one JSON line with the contract's keys, the roofline of the
local-reduce kernel and the CPU baselines.
N = 2: the path the driver's 8-GPU SCALE run takes (torchrun, one rank per GPU, ftar_init's
torchrun bootstrap, every leg of the N > 1 line), rehearsed with both ranks on GPU 0
(FTAR_DEVICE=0) and gloo for torch.distributed (RCCL refuses two ranks on one device),
at 4 MiB per rank so it runs in seconds.  The configs[4] leg runs as 5 ranks (4 + one
idle spare) because this box has one GPU.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


@pytest.mark.timeout(300)
def test_bench_single_gpu_line():
    # --no-pmc: the live counter passes (two rocprofv3 runs of a child) are the default bench's,
    # checked on the box by tools/gpu_check.sh's bench step; here the fallback's label is checked
    cp = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "2",
                         "--no-cpu-baseline", "--no-pmc"], capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert cp.returncode == 0, cp.stderr[-2000:]
    d = _last_json(cp.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "dtype", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 10 and d["roofline"]["bound"] == "hbm"
    # a fixed floor: 0.9 x the driver-observed 0.80 of 8 TB/s (boxes differ by a few %; the
    # kernel sits at the measured streaming ceiling)
    assert d["roofline"]["frac"] >= 0.72, d["roofline"]
    # without the live passes the PMC traffic is the committed figure, labelled with where it was
    # measured and why this run did not
    src = d["roofline"]["traffic_source"]
    assert src["measured_in_this_run"] is False and src["file"] == "profiles/pmc_summary.json", src
    assert src["live"] == {"measured_in_this_run": False, "skipped": "--no-pmc"}, src
    assert "rotating" in d["config"]["buffers"]


@pytest.mark.timeout(600)
def test_bench_two_rank_scale_path():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, FTAR_DEVICE="0", FTAR_C5_RANKS="5")
    for k in ("FTAR_JOB", "FTAR_RANK", "FTAR_SIZE", "FTAR_LAUNCHER", "FTAR_KILL"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--no-variants", "--count", str(1 << 20), "--steps", "2", "--warmup", "1",
           "--c5-draws", "3"]
    cp = subprocess.run(cmd, capture_output=True, text=True, timeout=540, cwd=ROOT, env=env)
    assert cp.returncode == 0, cp.stderr[-3000:]
    lines = [json.loads(l) for l in cp.stdout.splitlines() if l.startswith("{")]
    assert [x["line"] for x in lines] == ["headline", "final"], cp.stdout[-2000:]
    d = lines[-1]
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    ns = d["north_star"]  # present in a rehearsal too, fractions withheld (no link in the path)
    assert ns["rehearsal"] and ns["frac"] is None and ns["priced"]["survey_153.6_assumed"]["survey_t_roof_ms"] > 0
    assert all(v["status"] == "ok" for k, v in d["side_legs"].items() if isinstance(v, dict)), d["side_legs"]
    assert all(v["status"] == "ok" for v in d["legs"].values() if v["status"] != "skipped"), d["legs"]
    assert d["int32_rank_checksum_ok"] == {"raben": True, "rd": True}
    assert d["max_abs_err_vs_rccl"] < 1e-5
    ex = d["exact_on_node"]  # integer-valued float inputs, new per trial: bitwise exact
    assert ex["all_exact"] and ex["chosen"] and ex["reference_shape"] and ex["rd"] and ex["chosen_64KiB"], ex
    # every small-call mechanism on both sides of its threshold, gated and ungated
    for label in ("4B", "4KiB", "64KiB", "1MiB-16B", "1MiB", "1MiB+16B", "4MiB"):
        for algo in ("raben", "rd"):
            for g in ("gated", "ungated"):
                assert ex[f"{algo}_{label}_{g}"] is True, (algo, label, g, ex)
    assert "small_call_fallback" not in ex, ex
    assert d["size_sweep_us"] == {} or d["size_sweep_us"].get("small_call_setting", "").startswith("default")
    # the renamed north-star fields: the schedule's own bound, the reference's schedule, a speed-up
    for k in ("frac", "met", "reference_schedule_frac", "reference_schedule_met", "speedup_vs_survey_roofline",
              "frac_definition"):
        assert k in ns, (k, ns)
    assert d["config"]["schedule"] and d["config"]["transport"] == d["transport"]
    assert d["reference_shape"]["ms_per_step"] > 0
    cpu = d["cpu_baseline"]
    assert cpu and cpu["value"] and cpu["cores"] == 2 and cpu["kind"] == "port", cpu
    c5 = d["c5_single_kill"]
    assert c5 and c5["recovered"], c5
    kc = int(c5["kill"].split(" in call ")[1].split()[0])
    assert c5["fault"]["calls"][kc]["recoveries"] == 1 and c5["fault"]["survivors"] == 4
    assert all(c["result_ok"] for c in c5["no_fault"]["calls"]) and c5["survivors_call_ms"] > 0
    assert "mid-exchange" in c5["fault"].get("victim", ""), c5
    ref = c5["reference_shape"]  # the reference's recovery shape (FTAR_REDUNDANCY=1) recovers too
    assert ref["recovered"], ref
    # one GPU: the auto default elides the step-0 copy, the reference's shape moves it
    assert c5["no_fault"]["step0_copy"] == 0 and ref["no_fault"]["step0_copy"] == 1, (c5["no_fault"], ref["no_fault"])
    camp = c5["random_kill_campaign"]  # kill_procs.sh's random SIGKILL, seeded draws
    assert camp["draws_run"] == 3 and camp["wrong"] == 0 and camp["lost"] == 0, camp
    for rk in camp["runs"]:
        assert rk.get("killed") and rk["outcome"] in ("recovered", "aborted", "no fault hit") and \
            rk["results_consistent"], rk
    xg = d["xgmi_probe"]  # one GPU: the probe's kernels in loopback, destinations checked
    assert xg and xg["ok"] and "loopback_copy" in xg["patterns"], xg
    nd = d["node_decisions"]  # what the run decides, summarized in the line (analysis/analyze.py)
    assert "error" not in nd and nd["n_gpus"] == 2 and nd["rehearsal"] and nd["all_exact"], nd
