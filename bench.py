#!/usr/bin/env python3
"""bench.py -- Allreduce GB/s (device-resident, float32 SUM) of the MI355X-native
fault-tolerant Allreduce.

  python bench.py [--gpus 1] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

N = 1: the single-GPU workload of BASELINE.json configs[1] -- the local-reduce HIP
       kernel (MPI_Reduce_local, the per-step bucket reduction) on two 256 MiB float32
       vectors.  One step = one kernel launch.  HBM-bound.  The timed launches rotate
       over --pairs vector pairs (default 4 = 2 GiB) so no launch finds its operands in
       the 256 MiB Infinity Cache the previous launches filled: an HBM number.
N > 1: configs[3] -- fault-tolerant Rabenseifner Allreduce of a 256 MiB float32 vector
       per rank, one rank per GPU, exchanges pulled over xGMI (weak scaling: every rank
       contributes one 256 MiB vector).  One step = one Allreduce.  The schedule and
       transport that ran are named in `config`; the reference's own data movement
       (pairwise, step by step, step-0 full exchange) is timed as `reference_shape`.
       Recursive doubling (configs[2]), RCCL's all_reduce, a size sweep 4 B - 256 MiB
       (FT vs RCCL), the host-C CPU port of the schedule, and configs[4] (9 ranks = N
       GPUs + one idle spare, kills mid-exchange, recovery, a seeded random-kill
       campaign) are reported beside it.

The N > 1 run is built so that its first contact with a node cannot lose the headline:
  * the side legs (CPU baseline, fabric probe, configs[4] jobs) share ONE time budget
    (--side-budget) with a deadline per leg; a leg that overruns is killed (its own
    process group) and recorded as a timeout;
  * the headline JSON line is printed as soon as the configs[3] Allreduce is timed
    ("line": "headline"), with its roofline and north-star verdict; every later leg is
    optional, runs only while the job's budget (--budget) has room for it (decided
    uniformly over ranks), records its own failure, and the enriched line is printed last
    ("line": "final": the same keys plus the legs);
  * a watchdog prints what exists and ends the rank if the budget is overrun anyway.

value = (input vectors summed x bytes per vector) / time per step, whole job:
        N=1: 2 x 256 MiB per launch; N>1: N x 256 MiB per Allreduce.
Data are synthetic (uniform [-1, 1)), inputs resident in HBM before timing starts.
"""
import argparse
import importlib.util
import json
import os
import signal
import subprocess
import sys
import threading
import time

T_START = time.monotonic()
ROOT = os.path.dirname(os.path.abspath(__file__))
COUNT = 1 << 26              # 256 MiB of float32 per vector
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 76.8         # nominal: one xGMI link, one direction (153.6 GB/s bidirectional spec)
SURVEY_LINK_GBS = 153.6      # SURVEY.md 8d's nominal B_link "per direction" (assumption to confirm)
NORTH_STAR_FRAC = 0.70       # BASELINE.json north_star: >= 70 % of the xGMI-bound roofline at 8 GPUs
METRIC = "Allreduce GB/s (device-resident, float32 SUM) at 1/2/4/8 MI355X"
# data/data_fault/log_single_Raben.csv, N = 9, OK runs: median clock() seconds
REF_C5_S = {"kill": 1.334, "no_kill": 1.329, "count": 120732254}


class LegTimeout(RuntimeError):
    pass


def left(deadline):
    return deadline - time.monotonic()


def run_proc(cmd, timeout, env=None, cwd=None):
    """Run `cmd` in a session of its own and wait at most `timeout` s; past it the whole
    process group (the job's launcher and every rank it forked) is SIGKILLed.  Returns
    (rc, stdout, stderr, timed_out)."""
    p = subprocess.Popen(cmd, env=env, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=max(0.5, timeout))
        return p.returncode, out, err, False
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)  # the group this call created, nothing else
        except ProcessLookupError:
            pass
        out, err = p.communicate()
        return p.returncode, out, err, True


def test_hook(kind, leg):
    """TEST-ONLY fault hooks for the bench's own robustness tests (tests/test_bench_logic.py,
    tests/test_gpu_bench.py): FTAR_BENCH_HANG=<side leg> replaces that leg by a stand-in
    job that never ends; FTAR_BENCH_FAIL=<leg>[,<leg>...] makes that leg raise (on every
    rank at once).  Unset in every measured run."""
    v = os.environ.get("FTAR_BENCH_HANG" if kind == "hang" else "FTAR_BENCH_FAIL", "")
    return leg in [s.strip() for s in v.split(",") if s.strip()]


def maybe_hang(leg, deadline):
    if test_hook("hang", leg):
        rc, _, _, to = run_proc(["sleep", "3600"], left(deadline))
        if to:
            raise LegTimeout(f"{leg}: stand-in job still running at its deadline (killed)")


def maybe_fail(leg):
    if test_hook("fail", leg):
        raise RuntimeError(f"{leg}: forced failure (FTAR_BENCH_FAIL)")


def load_package():
    path = os.path.join(ROOT, "fault-tolerant_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("ftar_amd", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ftar_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_analysis():
    spec = importlib.util.spec_from_file_location(
        "ftar_analyze", os.path.join(ROOT, "fault-tolerant_amd", "analysis", "analyze.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def load_tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pmc_traffic(name):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_summary.json,
    written by tools/pmc_summary.py from separate `--pmc` passes), and where that number comes
    from: PMC counters need rocprofv3 around the process, so this run does not measure them --
    `traffic_source` names the file, the entry and the commit / date it was measured at."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    src = {"measured_in_this_run": False, "file": "profiles/pmc_summary.json", "entry": name}
    if not os.path.exists(path):
        return None, dict(src, missing=True)
    try:
        with open(path) as f:
            e = json.load(f).get(name, {})
    except (OSError, ValueError):
        return None, dict(src, unreadable=True)
    src.update({k: e[k] for k in ("measured_at", "command", "counters") if k in e})
    return e.get("hbm_bytes_per_launch"), src


def _under_profiler():
    """This process already runs under rocprofv3 (its preloaded library, its environment): a
    nested rocprofv3 would instrument the child twice, so the live counter passes are skipped."""
    pre = os.environ.get("LD_PRELOAD", "") + os.environ.get("HSA_TOOLS_LIB", "")
    return "rocprof" in pre or any(k.startswith("ROCPROF") for k in os.environ)


def pmc_live(args, kernel, steps=20, timeout=90.0):
    """HBM bytes per launch of the C2 kernel, measured in THIS run: two
    separate rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one pass) over
    a child `python3 bench.py --pmc-child` that launches the same kernel on the same rotating
    pairs, run before this process opens the GPU (a child is started, nothing is exec'ed; the
    profiled program is the child itself, right after `--`).  Corrected as MI355X_MICROARCH.md's
    HBM section prescribes for gfx950: 2 x FETCH_SIZE (half-counted 16-byte-per-lane streams) +
    WRITE_SIZE, KiB -> B, averaged over the kernel's dispatches.  Each pass is SIGKILLed with
    its process group past `timeout` (a counter request the hardware refuses hangs)."""
    import csv
    import shutil
    import tempfile
    rp = shutil.which("rocprofv3")
    if not rp or _under_profiler() or args.no_pmc:
        why = "no rocprofv3" if not rp else "--no-pmc" if args.no_pmc else "already under a profiler"
        return None, {"measured_in_this_run": False, "skipped": why}
    tmp = tempfile.mkdtemp(prefix="ftar_pmc_")
    vals, info = {}, {"measured_in_this_run": True, "counters": ["FETCH_SIZE", "WRITE_SIZE"], "passes": {}}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = [rp, "--pmc", ctr, "-d", d, "-o", "pmc", "--output-format", "csv", "--", sys.executable,
                   os.path.abspath(__file__), "--pmc-child", "--steps", str(steps), "--count", str(args.count),
                   "--pairs", str(args.pairs), "--variant", str(args.variant)]
            t0 = time.monotonic()
            rc, out, err, to = run_proc(cmd, timeout)
            info["passes"][ctr] = {"rc": rc, "s": round(time.monotonic() - t0, 1), "timed_out": to}
            files = [os.path.join(r, n) for r, _, fs in os.walk(d) for n in fs if n.endswith("counter_collection.csv")]
            v = []
            for fp in files:
                with open(fp, newline="") as f:
                    v += [float(row["Counter_Value"]) for row in csv.DictReader(f)
                          if row["Counter_Name"] == ctr and kernel in row["Kernel_Name"]]
            if rc != 0 or to or not v:
                info["error"] = f"{ctr}: rc {rc}, timed out {to}, {len(v)} dispatches; {err[-300:]}"
                return None, info
            vals[ctr] = (sum(v) / len(v), len(v))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    info.update({"kernel": kernel, "dispatches": [vals["FETCH_SIZE"][1], vals["WRITE_SIZE"][1]],
                 "FETCH_SIZE_KiB": round(vals["FETCH_SIZE"][0], 1), "WRITE_SIZE_KiB": round(vals["WRITE_SIZE"][0], 1),
                 "correction": "2*FETCH_SIZE (gfx950 half-count on 16B/lane streams) + WRITE_SIZE, KiB->B"})
    return round((2 * vals["FETCH_SIZE"][0] + vals["WRITE_SIZE"][0]) * 1024), info


def pmc_child(args):
    """The profiled child of pmc_live: the C2 kernel on the bench's rotating pairs, nothing else."""
    import torch
    ftar = load_package()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(42)
    pairs = [(torch.rand(args.count, device="cuda", generator=g), torch.rand(args.count, device="cuda", generator=g))
             for _ in range(args.pairs)]
    ftar.set_reduce_variant(args.variant)
    torch.cuda.synchronize()
    for k in range(args.steps):
        x, y = pairs[k % args.pairs]
        ftar.reduce_local(x, y)
    torch.cuda.synchronize()


def cpu_baseline_local_reduce(min_seconds=10.0, max_passes=2000):
    """The oracle's MPI_Reduce_local restatement on the host (1 thread), same workload."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rng = np.random.default_rng(1)
    a = rng.random(COUNT, dtype=np.float32)
    b = rng.random(COUNT, dtype=np.float32)
    O.reduce_local(a, b)  # warm the pages
    t0 = time.perf_counter()
    passes = 0
    while passes < max_passes and (time.perf_counter() - t0) < min_seconds:
        O.reduce_local(a, b)
        passes += 1
    dt = time.perf_counter() - t0
    return {"value": round(2 * COUNT * 4 * passes / dt / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"oracle/ftar_oracle.c reduce_local, 2 x 256 MiB float32, {passes} passes "
                      f"({dt:.1f} s), 1 host thread"}


def cpu_schedule(algo, p, count, reps, timeout=600.0):
    """The schedule on the host cores: the product's host C (control plane, agree rounds,
    the FT schedule) as p processes pinned one per core, POSIX shared memory as the
    transport, C loops as the reduce (tools/cpu_schedule_bench.py), float32."""
    cs = load_tool("cpu_schedule_bench")
    cs.build()
    r = cs.run(algo, p, count, "float32", reps, timeout=timeout)
    return r, cs.cpu_model()


def c1_baseline(timeout=120.0):
    """BASELINE configs[0]: src/rd/main recursive doubling, float32 SUM, 64 KiB, 4 ranks."""
    r, model = cpu_schedule("rd", 4, 16384, 20, timeout=timeout)
    return {"value": round(4 * 16384 * 4 / r["time_s"] / 1e9, 4), "unit": "GB/s", "ms_per_call": round(r["time_s"] * 1e3, 4),
            "algbw_GBps": r["algbw_GBps"], "cores": 4, "kind": "port", "cpu_model": model,
            "sample": "configs[0]: recursive doubling, 64 KiB float32 SUM per rank, 4 rank processes pinned one "
                      "per core, pairwise step-by-step exchanges through shared memory, median of 20 runs "
                      "(value = 4 x 64 KiB / call time, as the GPU lines)",
            "reference_leonardo_ms": 0.976}


def single(args):
    # the counter passes first, while this process has not opened the GPU (their child is a
    # GPU process of its own)
    kname = "reduce_lds_kernel" if args.variant == 1 else "segment_kernel"
    live_traffic, live_src = pmc_live(args, kname)
    import torch
    ftar = load_package()
    ftar.lib()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(42)
    pairs = [(torch.rand(args.count, device="cuda", generator=g) * 2 - 1,
              torch.rand(args.count, device="cuda", generator=g) * 2 - 1) for _ in range(args.pairs)]
    ftar.set_reduce_variant(args.variant)
    for k in range(args.warmup):
        x, y = pairs[k % args.pairs]
        ftar.reduce_local(x, y)
    torch.cuda.synchronize()

    def region(steps, npairs):
        # one event pair around the whole timed region, on the stream the kernels run on
        # (torch's current stream, which reduce_local launches on): the average launch
        # duration includes the kernel-to-kernel boundaries, nothing runs in between
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for k in range(steps):
            x, y = pairs[k % npairs]
            ftar.reduce_local(x, y)
        e1.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        return (t1 - t0) * 1e3 / steps, e0.elapsed_time(e1) / steps

    if args.timing == "launch":
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        t0 = time.perf_counter()
        for k, (e0, e1) in enumerate(evs):
            x, y = pairs[k % args.pairs]
            e0.record()
            ftar.reduce_local(x, y)
            e1.record()
        torch.cuda.synchronize()
        ms_step = (time.perf_counter() - t0) * 1e3 / args.steps
        k_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / args.steps
    else:
        ms_step, k_ms = region(args.steps, args.pairs)
    # the same launches on ONE pair (operands partly left in the Infinity Cache by the
    # previous launch): what round 1 timed; reported, not the headline
    _, k_same = region(min(args.steps, 100), 1)
    S = args.count * 4
    achieved = 3 * S / (k_ms * 1e-3) / 1e9
    if live_traffic:
        traffic, traffic_src = live_traffic, live_src
    else:  # the committed figure, labelled as such (and why this run did not measure it)
        traffic, traffic_src = pmc_traffic("reduce_local_c2_lds_rot" if args.variant == 1 else "reduce_local_c2_rot")
        traffic_src["live"] = live_src
    out = {
        "metric": METRIC, "value": round(2 * S / (ms_step * 1e-3) / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic uniform[-1,1), HBM-resident",
        "config": {"workload": "configs[1]: local-reduce HIP kernel (MPI_Reduce_local), 2 x 256 MiB float32 SUM, "
                               "1 MI355X", "count": args.count, "kernel_variant": args.variant,
                   "timing": args.timing,
                   "buffers": f"{args.pairs} rotating pairs ({args.pairs * 2 * S >> 20} MiB working set, "
                              f"beyond the 256 MiB Infinity Cache)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_over_algorithmic": round(traffic / (3 * S), 5) if traffic else None,
                     "kernel": "reduce_lds_kernel<float,SUM>" if args.variant == 1 else "segment_kernel<float,SUM>",
                     "algorithmic_bytes_per_launch": 3 * S,
                     "kernel_ms": round(k_ms, 4),
                     "same_pair_kernel_ms": round(k_same, 4),
                     "same_pair_GBps": round(3 * S / (k_same * 1e-3) / 1e9, 1)},
    }
    out["e2e"] = e2e_local(ftar, args.count, args.variant)
    if args.no_cpu_baseline:
        out["cpu_baseline"] = None
    else:
        out["cpu_baseline"] = cpu_baseline_local_reduce()
        try:
            out["cpu_baseline"]["c1"] = c1_baseline()
        except Exception as e:  # reported, never fatal: the GPU line stands on its own
            out["cpu_baseline"]["c1"] = {"error": str(e)[-300:]}
    print(json.dumps(out), flush=True)


def e2e_local(ftar, count, variant, iters=5):
    """Host-resident variant of the same step: pinned H2D of both vectors, the kernel,
    pinned D2H of the result (PCIe-bound), never the headline value."""
    import torch
    xh = torch.rand(count).pin_memory()
    yh = torch.rand(count).pin_memory()
    xd = torch.empty(count, device="cuda")
    yd = torch.empty(count, device="cuda")
    S = count * 4
    ts = {"h2d": 0.0, "d2h": 0.0, "total": 0.0}
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        xd.copy_(xh, non_blocking=True)
        yd.copy_(yh, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ftar.reduce_local(xd, yd)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        yh.copy_(yd, non_blocking=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ts["h2d"] += t1 - t0
        ts["d2h"] += t3 - t2
        ts["total"] += t3 - t0
    out = {"h2d_GBps": round(2 * S * iters / ts["h2d"] / 1e9, 2), "d2h_GBps": round(S * iters / ts["d2h"] / 1e9, 2),
           "ms": round(ts["total"] * 1e3 / iters, 3),
           "GBps": round(2 * S * iters / ts["total"] / 1e9, 2)}
    # zero copy: the kernel reads both pinned host vectors and writes the result back
    # over PCIe in one pass -- reads and writes on the link's two directions at once
    # instead of H2D, kernel, D2H in turn (ftar_reduce_local accepts pinned host memory)
    # (the register kernel, as fast here: the 10 ms PCIe-bound launches then stay out of
    # the headline kernel's rocprof statistics)
    y0 = torch.rand(count)
    tz = 0.0
    ftar.set_reduce_variant(0)
    for _ in range(iters):
        yh.copy_(y0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ftar.reduce_local(xh, yh)
        torch.cuda.synchronize()
        tz += time.perf_counter() - t0
    ftar.set_reduce_variant(variant)
    out["zero_copy"] = {"ms": round(tz * 1e3 / iters, 3), "GBps": round(2 * S * iters / tz / 1e9, 2),
                        "pcie_GBps": round(3 * S * iters / tz / 1e9, 2),
                        "exact": bool(torch.equal(yh, y0 + xh))}
    return out


# ---- configs[4]: its own ftrun jobs (torchrun's agent tears a job down on a SIGKILL) ----

def _c5_env():
    return {k: v for k, v in os.environ.items()
            if not k.startswith(("FTAR_", "RANK", "LOCAL_", "WORLD_", "GROUP_", "ROLE_", "TORCHELASTIC"))}


def _ftrun_paths():
    return (os.path.join(ROOT, "fault-tolerant_amd", "bin", "ftrun"),
            os.path.join(ROOT, "fault-tolerant_amd", "bin", "ftbench"))


def _mid_exchange_lines(stderr):
    """ftrun's post-mortem of every rank killed by a signal (the victim's control slot: was a
    kernel of its exchange in flight when it died?) and the DURING victim's own line."""
    return [l.split("ftrun: ")[-1] if "ftrun: " in l else l.split("ftar: ")[-1]
            for l in stderr.splitlines() if "mid-exchange" in l or "killed by signal" in l]


def c5_leg(world, devices, count, ranks, deadline, calls=6, kill_call=2):
    """configs[4] on this node: `ranks` = world GPUs' worth of ranks + one idle spare (rank
    1 shares rank 0's GPU), Rabenseifner 256 MiB float32 SUM, `calls` calls per job; the
    fault job kills vrank 5 (original rank 6) in reduce-scatter step 1 of call `kill_call`,
    mid-exchange (its own pull kernel in flight, its partner's pull reading its HBM), a
    second one in allgather step 1 ("also AG step 1"; the last AG step when
    there are only two).  Every job runs in both recovery shapes: the library's default
    (FTAR_REDUNDANCY auto: the reference's step-0 copy moves when the ranks span more than
    one GPU, raben/rabenseifner.c:206-211; on one GPU it is elided and the replay reads the
    dead rank's step-0 half in its still-mapped IN, DESIGN.md deviation 6) and the other one
    (on the node the elided shape, opt-in FTAR_REDUNDANCY=0 -- its RS-kill job says whether a
    dead process's memory stays readable across GPUs: `dead_input_cross_device`; on one GPU
    the reference's copy, FTAR_REDUNDANCY=1).  The recovery shrinks the comm; the later
    calls run on the survivors.  Call 0 is the warm-up (workspace allocation, IPC
    imports).  Every job ends by `deadline` (killed past it)."""
    ftrun, exe = _ftrun_paths()
    devmap = [devices[0], devices[0]] + [devices[(r - 1) % len(devices)] for r in range(2, ranks)]
    victim = 6 if ranks > 6 else ranks - 1
    ag_step = 1 if ranks >= 8 else 0  # a middle allgather step where there is one (L >= 3)
    env = _c5_env()
    multi_gpu = len(set(devmap)) > 1
    res = {"ranks": ranks, "devmap": devmap, "count": count, "calls": calls,
           "kill": f"{victim}:1:1:3 in call {kill_call} (original rank {victim} = vrank {victim - 1}, reduce-scatter "
                   "step 1, mid-exchange)",
           "kill_ag": f"{victim}:2:{ag_step}:3 in call {kill_call} (allgather step {ag_step}, mid-exchange)"}
    want_all = float(sum(range(ranks)))

    def job(kill, redundancy):
        e = dict(env)
        if kill:
            e["FTAR_KILL"] = kill
        if redundancy is not None:
            e["FTAR_REDUNDANCY"] = redundancy
        t0 = time.time()
        rem = left(deadline)
        if rem < 1.0:
            return {"skipped": "side-leg budget spent"}
        rc, out, err, to = run_proc([ftrun, "-np", str(ranks), "--devmap", ",".join(map(str, devmap)), exe, "raben",
                                     str(count), str(calls)], min(rem, 120.0), env=e)
        lines = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
        per_call = []
        for c in range(calls):
            per = [ln["calls"][c] for ln in lines]
            # the kill call still sums every input (the dead rank's block is recovered,
            # the reference's corr path); later calls sum the survivors'
            want = want_all - (victim if (kill and c > kill_call) else 0)
            per_call.append({"ms_max_over_ranks": round(max(p["ms"] for p in per), 3) if per else None,
                             # algorithmic local HBM bytes of the busiest rank's kernels (ftar_stats.hbm_bytes)
                             "hbm_bytes_max_over_ranks": max((p.get("hbm_bytes", 0) for p in per), default=None),
                             "recoveries": max((p["recoveries"] for p in per), default=None),
                             "comm_size_after": min((p["comm_size"] for p in per), default=None),
                             "result_ok": bool(per) and all(p["rc"] == 0 and p["uniform"] and p["value"] == want
                                                            for p in per)})
        r = {"rc": rc, "survivors": len(lines), "job_wall_s": round(time.time() - t0, 2), "calls": per_call,
             "aborted": "MPI_ABORT" in err,
             "device_error": any(s in err for s in ("device error", "Memory access fault", "HSA_STATUS_ERROR")),
             "step0_copy": lines[0].get("step0_copy") if lines else None}
        if to:
            r["timed_out"] = True
        if rc != 0 or not lines:
            r["stderr_tail"] = err[-600:]
        mid = [l for l in err.splitlines() if "dies mid-exchange" in l]
        if mid:
            r["victim"] = mid[0].split("ftar: ")[-1]
        return r

    def med(cs):
        v = sorted(c["ms_max_over_ranks"] for c in cs if c["ms_max_over_ranks"] is not None)
        return v[len(v) // 2] if v else None

    def recovered(j):
        fc = j.get("calls")
        return bool(fc) and j["survivors"] == ranks - 1 and fc[kill_call]["recoveries"] == 1 and \
            all(c["result_ok"] for c in fc)

    def summarize(n, f, fa):
        s = {}
        try:
            s["recovered_rs"] = recovered(f)
            s["recovered_ag"] = recovered(fa)
            s["recovered"] = s["recovered_rs"] and s["recovered_ag"]
            fc = f["calls"]
            s["recovered_call_ms"] = fc[kill_call]["ms_max_over_ranks"]
            s["recovered_ag_call_ms"] = fa["calls"][kill_call]["ms_max_over_ranks"]
            s["no_fault_call_ms"] = med(n["calls"][1:])  # median after the warm-up call
            s["no_fault_hbm_bytes"] = n["calls"][-1].get("hbm_bytes_max_over_ranks")
            s["recovery_overhead_ms"] = round(s["recovered_call_ms"] - s["no_fault_call_ms"], 3)
            s["pre_fault_call_ms"] = med(fc[1:kill_call])
            s["survivors_call_ms"] = med(fc[kill_call + 1:])  # p - 1 ranks after the shrink
        except (KeyError, IndexError, TypeError, ValueError):
            s["recovered"] = False
        return s

    maybe_hang("c5", deadline)
    jobs = (("no_fault", None), ("fault", f"{victim}:1:1:3:{kill_call}"), ("fault_ag", f"{victim}:2:{ag_step}:3:{kill_call}"))
    for name, kill in jobs:
        res[name] = job(kill, None)
    res.update(summarize(res["no_fault"], res["fault"], res["fault_ag"]))
    copy_desc = ("the reference's step-0 copy of the partner's other half moves in every call and the RS replay reads "
                 "it (raben/rabenseifner.c:206-211, raben/errhandler.c:106-200)")
    elided_desc = ("no step-0 copy; the RS replay reads the dead rank's step-0 half in its IN, still mapped by the "
                   "peers (DESIGN.md 3, deviation 6)")
    res["recovery_shape"] = ("default (FTAR_REDUNDANCY auto): " + (copy_desc + " -- the ranks span GPUs" if multi_gpu
                                                                   else elided_desc + " -- one GPU"))
    other = {"shape": ("FTAR_REDUNDANCY=0 (opt-in): " + elided_desc) if multi_gpu else
             ("FTAR_REDUNDANCY=1: " + copy_desc)}
    for name, kill in jobs:
        other[name] = job(kill, "0" if multi_gpu else "1")
    other.update(summarize(other["no_fault"], other["fault"], other["fault_ag"]))
    if multi_gpu:
        # the premise of the elided shape, decided on the node: does a SIGKILLed rank's
        # memory stay readable through its peers' mappings across GPUs?
        f = other["fault"]
        other["dead_input_cross_device"] = ("recovered" if other.get("recovered_rs") else "abort" if f.get("aborted")
                                            else "fault" if f.get("device_error") or f.get("rc") else "wrong")
        res["elided_shape"] = other
        res["dead_input_cross_device"] = other["dead_input_cross_device"]
    else:
        res["reference_shape"] = other
    res["reference_leonardo_s"] = dict(REF_C5_S, note="clock() s per run incl. the whole MPI job, 460.6 MiB int32")
    return res


def reference_outcomes(n):
    """The reference's recorded single-kill outcomes at N = n (tests/golden/ref_fault_outcomes.csv,
    from data/data_fault/log_single_Raben.csv): recovered / MPI_Abort / deadlock."""
    path = os.path.join(ROOT, "tests", "golden", "ref_fault_outcomes.csv")
    out = {"recovered": 0, "aborted": 0, "deadlock": 0, "wrong": 0,
           "source": "data/data_fault/log_single_Raben.csv via tests/golden/ref_fault_outcomes.csv"}
    try:
        for line in open(path).read().splitlines()[1:]:
            algo, N, killed, abort, dead, right, cnt = line.split(";")
            if algo != "raben" or int(N) != n or int(killed) == 0:
                continue
            if abort == "True":
                out["aborted"] += int(cnt)
            elif dead == "True":
                out["deadlock"] += int(cnt)
            elif right == "True":
                out["recovered"] += int(cnt)
            else:
                out["wrong"] += int(cnt)
    except (OSError, ValueError):
        return None
    return out


def c5_random_kill(ftrun, exe, ranks, devmap, count, env, deadline, calls=3, loop_s=1.5, seed=0):
    """One draw of the reference's random kill (run/kill_procs.sh: SIGKILL one rank process
    after a random delay) on the configs[4] job.  Each call is stretched to `loop_s` seconds
    (FTAR_LOOP_SECONDS, as run/run_mpi.sh does) with idempotent re-pulls of the step's
    window, so the kill lands while exchange kernels are in flight; ftrun's post-mortem
    says whether the victim died with one in flight.  The outcome is the reference's
    (recovered, or MPI_Abort where its handler aborts), and every survivor's results must
    agree, call by call, on the exact sum with or without the victim's input, never
    dropping it and taking it back."""
    import random
    rng = random.Random(seed)
    victim = rng.randrange(ranks)
    delay = rng.uniform(1.5, 1.0 + loop_s * calls)  # after the launch: ~1 s of process start-up
    e = dict(env, FTAR_LOOP_SECONDS=str(loop_s))
    out = {"seed": seed, "victim": victim, "delay_s": round(delay, 3), "loop_seconds": loop_s, "calls": calls}
    pr = None
    try:
        import psutil
        t0 = time.time()
        pr = subprocess.Popen([ftrun, "-np", str(ranks), "--devmap", ",".join(map(str, devmap)), exe, "raben",
                               str(count), str(calls)], env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, start_new_session=True)
        time.sleep(min(delay, max(0.0, left(deadline) - 1.0)))
        for k in psutil.Process(pr.pid).children():  # the rank processes ftrun started
            try:
                if k.environ().get("FTAR_RANK") == str(victim):
                    os.kill(k.pid, signal.SIGKILL)
                    out["killed"] = True
            except (psutil.Error, OSError):
                pass
        so, se = pr.communicate(timeout=max(1.0, min(60.0, left(deadline))))
        out["job_wall_s"] = round(time.time() - t0, 2)
        out["rc"] = pr.returncode
    except subprocess.TimeoutExpired:
        os.killpg(pr.pid, signal.SIGKILL)
        pr.communicate()
        out["outcome"] = "lost"
        out["error"] = "job still running at its deadline (deadlock?): killed"
        return out
    except Exception as ex:
        out["error"] = str(ex)[-300:]
        out["outcome"] = "error"
        if pr is not None and pr.poll() is None:
            os.killpg(pr.pid, signal.SIGKILL)
            pr.wait()
        return out
    lines = [json.loads(l) for l in so.splitlines() if l.startswith("{")]
    full = float(sum(range(ranks)))
    out["aborted"] = "MPI_ABORT" in se
    out["survivors"] = len(lines)
    out["post_mortem"] = _mid_exchange_lines(se)
    out["mid_exchange"] = any("killed by signal" in l and "mid-exchange" in l for l in out["post_mortem"])
    consistent = bool(lines) or out["aborted"]
    dropped = False
    per = []
    for c in range(calls):
        vals = {ln["calls"][c]["value"] for ln in lines}
        ok = len(vals) <= 1 and all(ln["calls"][c]["rc"] == 0 and ln["calls"][c]["uniform"] for ln in lines)
        v = vals.pop() if len(vals) == 1 else None
        if v is not None and v not in (full, full - victim):
            ok = False
        if dropped and v == full and victim != 0:  # (rank 0's input is 0: both sums coincide)
            ok = False
        dropped = dropped or v == full - victim
        consistent = consistent and ok
        per.append({"value": v, "recoveries": max((ln["calls"][c]["recoveries"] for ln in lines), default=None),
                    "ms_max_over_ranks": round(max((ln["calls"][c]["ms"] for ln in lines), default=0.0), 3)})
    out["per_call"] = per
    out["results_consistent"] = consistent
    if not lines and not out["aborted"]:
        # no survivor printed and nobody called MPI_Abort: the job itself failed
        out["outcome"] = "failed"
        out["stderr_tail"] = se[-400:]
    elif not consistent:
        out["outcome"] = "wrong"
        out["ranks_calls"] = [[(c["rc"], c["value"], c["uniform"], c["recoveries"], c["comm_size"]) for c in ln["calls"]]
                              for ln in lines]
        out["stderr_tail"] = se[-1500:]
    else:
        out["outcome"] = "aborted" if out["aborted"] else "recovered" if len(lines) == ranks - 1 else \
            "no fault hit" if len(lines) == ranks else "lost"
    return out


def c5_campaign(devices, count, ranks, deadline, draws=10, seed0=0):
    """configs[4]'s random-kill campaign: up to `draws` seeded draws (victim, delay) of
    c5_random_kill at `ranks` ranks while the side-leg budget lasts, with the outcome counts
    next to the reference's own at N = 9."""
    ftrun, exe = _ftrun_paths()
    devmap = [devices[0], devices[0]] + [devices[(r - 1) % len(devices)] for r in range(2, ranks)]
    maybe_hang("c5_campaign", deadline)
    runs = []
    for k in range(draws):
        if left(deadline) < 9.0:  # a draw takes ~5-7 s: start none that cannot finish
            break
        runs.append(c5_random_kill(ftrun, exe, ranks, devmap, count, _c5_env(), deadline, seed=seed0 + k))
    counts = {}
    for r in runs:
        counts[r.get("outcome", "error")] = counts.get(r.get("outcome", "error"), 0) + 1
    killed = [r for r in runs if r.get("killed")]
    return {"ranks": ranks, "count": count, "draws_planned": draws, "draws_run": len(runs), "outcomes": counts,
            "mid_exchange_kills": sum(1 for r in killed if r.get("mid_exchange")), "kills": len(killed),
            "wrong": counts.get("wrong", 0), "lost": counts.get("lost", 0),
            "reference_single_kill_N9": reference_outcomes(9), "runs": runs}


def leg_flag(tag):
    """Flag file rank 0 writes when a rank-0 leg ends (one per torchrun job: its master
    port and agent pid)."""
    return os.path.join("/tmp", f"ftar-bench-{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}-{tag}")


def side_legs(args, rank, world, devices, rehearsal):
    """The legs rank 0 runs as other processes -- the CPU baseline (host processes), the
    fabric probe (one process on every GPU) and the configs[4] jobs (ftrun, 9 ranks) --
    BEFORE any torchrun rank touches a GPU: the other ranks wait here on a flag file
    (importing torch opens no GPU: tools/kfd_probe.py).  Run after the main legs they would
    share the cards with the job's own ranks (8 + 9 GPU processes at N = 8, beyond what a
    box lets one job run on a card).  All of them share ONE budget (args.side_budget s):
    each leg gets a deadline carved out of what is left, a leg past its deadline is killed
    and recorded, and the flag is written whatever happens.  Returns (cpu, c5, xgmi, info)
    on rank 0, Nones elsewhere."""
    flag = leg_flag("side")
    if rank != 0:
        limit = time.monotonic() + args.side_budget + 60.0
        while not os.path.exists(flag) and time.monotonic() < limit:
            time.sleep(0.05)
        return None, None, None, None
    S = args.count * 4
    cpu = c5 = xgmi = None
    end = time.monotonic() + args.side_budget
    info = {"budget_s": args.side_budget}

    def leg(name, share, fn):
        d = min(end, time.monotonic() + share * args.side_budget)
        t0 = time.monotonic()
        try:
            if left(d) < 1.0:
                raise LegTimeout("no budget left")
            r = fn(d)
            status = "ok"
        except LegTimeout as e:
            r, status = {"error": str(e)[-300:]}, "timeout"
        except Exception as e:  # recorded, never fatal: the line stands without this leg
            r, status = {"error": str(e)[-500:]}, "error"
        info[name] = {"status": status, "s": round(time.monotonic() - t0, 2), "deadline_s": round(d - t0, 1)}
        return r

    def cpu_leg(d):
        # the same schedule on this node's host cores, float32, 256 MiB per rank
        maybe_hang("cpu_baseline", d)
        r, model = cpu_schedule("raben", world, args.count, 3, timeout=left(d))
        return {"value": round(world * S / r["time_s"] / 1e9, 4), "unit": "GB/s", "cores": world,
                "kind": "port", "cpu_model": model, "ms_per_call": round(r["time_s"] * 1e3, 2),
                "algbw_GBps": r["algbw_GBps"],
                # the reference's TIME is clock() of one rank: CPU seconds per rank
                # process (ranks spin, so it tracks wall time; it also covers init,
                # fill, checksum)
                "cpu_s_per_rank_process": r["cpu_s_per_rank_whole_process"],
                "sample": f"Rabenseifner (FT, the reference's step-by-step pairwise shape), {world} rank "
                          f"processes pinned one per core, 256 MiB float32 per rank through shared memory, "
                          f"median of 3 calls (driver Time: lines, max over ranks); value = {world} x 256 MiB "
                          f"/ call time"}

    def xgmi_leg(d):
        # the fabric (tools/xgmi_probe.hip, one process driving the job's GPUs): one link
        # one way and both ways (SURVEY.md 8d's B_link), pull vs push, copy engines, the
        # mesh's all-peers pattern; loopback in a one-GPU rehearsal
        maybe_hang("xgmi_probe", d)
        exe = os.path.join(ROOT, "tools", "_build", "xgmi_probe")
        rc, out, err, to = run_proc([exe, str(1 if rehearsal else world)], left(d))
        if to:
            raise LegTimeout("xgmi_probe still running at its deadline (killed)")
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        return json.loads(lines[-1]) if lines else {"error": (err or out)[-300:], "rc": rc}

    try:
        if not args.no_cpu_baseline:
            cpu = leg("cpu_baseline", 0.2, cpu_leg)
            if "error" in cpu:
                cpu = {"value": None, "unit": "GB/s", "cores": world, "kind": "port",
                       "sample": f"failed: {cpu['error']}"}
        if not args.no_xgmi:
            xgmi = leg("xgmi_probe", 0.2, xgmi_leg)
        if not args.no_c5:
            # configs[4]: N GPUs' worth of ranks + the idle spare, its own ftrun jobs
            ranks = int(os.environ.get("FTAR_C5_RANKS", "9"))
            c5 = leg("c5", 0.35, lambda d: c5_leg(world, devices, args.count, ranks, d))
            camp = leg("c5_campaign", 1.0, lambda d: c5_campaign(devices, args.count, ranks, d,
                                                                 draws=args.c5_draws))
            if isinstance(c5, dict):
                c5["random_kill_campaign"] = camp
    finally:
        info["total_s"] = round(args.side_budget - left(end), 2)
        with open(flag, "w") as f:
            f.write("done")
    return cpu, c5, xgmi, info


class Watchdog(threading.Thread):
    """Last resort against a hang the per-leg deadlines cannot reach (a collective stuck
    on one rank): at `limit` s after the start rank 0 prints the line as it stands
    ("truncated") and every rank exits.  Rank 0 fires first so it prints before a peer's
    exit can abort the job."""

    def __init__(self, limit, rank):
        super().__init__(daemon=True)
        self.limit = limit + (0.0 if rank == 0 else 5.0)
        self.rank = rank
        self.line = None
        self.done = threading.Event()

    def run(self):
        if self.done.wait(max(0.0, self.limit - (time.monotonic() - T_START))):
            return
        if self.rank == 0 and self.line is not None:
            d = dict(self.line, line="final", truncated=f"watchdog: the job passed its {self.limit:.0f} s budget; "
                                                        "legs missing here did not finish")
            print(json.dumps(d), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if self.line is not None else 3)


def _fraction(bound_s, t_s):
    """A roofline fraction: the time bound over the measured time.  Above 1 (beyond timer
    noise) the measurement beat its own bound -- the link price underestimates the fabric --
    so no fraction is claimed: `frac` is null, the ratio is kept as `frac_raw`, `met` null."""
    r = bound_s / t_s
    if r > 1.02:
        return {"frac": None, "frac_raw": round(r, 4), "met": None,
                "bound_violated": "measured time below this bound: the link price is too low (see link_calibration)"}
    return {"frac": round(r, 4), "met": r >= NORTH_STAR_FRAC}


def north_star_block(world, S, t_head, transport, link_gbps, links, head_bytes_per_link, t_ref=None, rehearsal=False,
                     breakdown=None):
    """BASELINE.json north_star / SURVEY.md 8d: >= 70 % of the xGMI-bound roofline for the
    device-resident Rabenseifner Allreduce of 256 MiB float32 at 8 GPUs.

    Every `frac` here is a time bound divided by the time of the schedule it bounds:
      * `frac` / `met` (top level): the timed headline schedule against ITS OWN link bound --
        e.g. the one-hop mesh moves 2 S / p over each of p - 1 links at once, so its bound
        is (2 S / p) / B_link -- at the calibrated single-link rate B_link (both directions
        loaded), the nominal 76.8 / SURVEY's 153.6 GB/s per direction beside it as assumptions;
      * `reference_schedule_frac`: the reference's own data movement (pairwise, step by step,
        step-0 full exchange: (2.5 - 2^(1-L)) S per rank and direction over one link per step,
        2.25 S at p = 8 -- SURVEY.md 8d's roofline) timed in the same job, against that bound;
      * `speedup_vs_survey_roofline`: SURVEY's FT roofline time over the headline time -- how
        much faster the schedule that ran is than the reference's schedule could ever be on
        one link per step.  A speed-up, never a fraction: it exceeds 1 by design;
      * `non_kernel_ms` (from `breakdown`, the profiled pass of the headline): the call's time
        outside its kernels -- host drains, agree + barrier rounds, launch latency -- beside
        `kernels_ms`, and `frac_kernels_only`: the schedule's bound over the kernels' time, the
        fraction the call would reach with no time outside kernels (at
        the 70 % target, 1.25 ms per call, every 0.1 ms outside kernels costs ~6 points)."""
    L = world.bit_length() - 1
    ft_bytes = (2.5 - 2.0 ** (1 - L)) * S
    priced = {}
    for tag, b in (("calibrated", link_gbps), ("nominal_76.8_assumed", XGMI_LINK_GBS),
                   ("survey_153.6_assumed", SURVEY_LINK_GBS)):
        if not b:
            continue
        t_roof = ft_bytes / (b * 1e9)
        t_sched = head_bytes_per_link / (b * 1e9)
        row = {"link_GBps": round(b, 2), "schedule_t_roof_ms": round(t_sched * 1e3, 4),
               "schedule": _fraction(t_sched, t_head),
               "survey_t_roof_ms": round(t_roof * 1e3, 4), "survey_algbw_roof_GBps": round(S / t_roof / 1e9, 2),
               "survey_target_algbw_GBps": round(NORTH_STAR_FRAC * S / t_roof / 1e9, 2),
               "speedup_vs_survey_roofline": round(t_roof / t_head, 4)}
        if t_ref:
            row["reference_schedule"] = _fraction(t_roof, t_ref)
        priced[tag] = row
    basis = "calibrated" if "calibrated" in priced else "survey_153.6_assumed"
    if rehearsal:  # every rank on one GPU: no link in the path, fractions would mix yardsticks
        for row in priced.values():
            row["schedule"] = {"frac": None, "met": None}
            row["speedup_vs_survey_roofline"] = None
            if "reference_schedule" in row:
                row["reference_schedule"] = {"frac": None, "met": None}
    b = priced[basis]
    out = {"target": f">= {NORTH_STAR_FRAC:.0%} of the xGMI-bound roofline, FT Rabenseifner, 256 MiB float32 SUM, "
                     f"8 GPUs", "applies": world == 8, "n_gpus": world,
           "frac_definition": "headline schedule's own link bound / its measured time (bytes per link / B_link)",
           "schedule": transport, "schedule_bytes_per_link": head_bytes_per_link, "schedule_links": links,
           "algbw_GBps": round(S / t_head / 1e9, 2), "ms_per_step": round(t_head * 1e3, 4),
           "basis": basis, "frac": b["schedule"]["frac"], "met": b["schedule"]["met"],
           "survey_roofline_definition": f"(2.5 - 2^(1-L)) S = {ft_bytes:.0f} B per rank and direction over one link "
                                         "per step (the reference's FT schedule), at B_link",
           "speedup_vs_survey_roofline": b["speedup_vs_survey_roofline"],
           "priced": priced, "rehearsal": rehearsal}
    if "bound_violated" in b["schedule"]:
        out["bound_violated"] = b["schedule"]["bound_violated"]
    if t_ref:
        out["reference_shape_ms"] = round(t_ref * 1e3, 4)
        out["reference_schedule_frac"] = b["reference_schedule"]["frac"]
        out["reference_schedule_met"] = b["reference_schedule"]["met"]
    if breakdown and breakdown.get("call_ms") is not None and breakdown.get("kernels_ms") is not None:
        call_ms, kern_ms = breakdown["call_ms"], breakdown["kernels_ms"]
        nk = max(0.0, call_ms - kern_ms)
        out["call_ms_profiled"] = call_ms
        out["kernels_ms"] = kern_ms
        out["non_kernel_ms"] = round(nk, 4)
        out["non_kernel_share"] = round(nk / call_ms, 4) if call_ms > 0 else None
        out["non_kernel_parts_ms"] = {"agree_barrier_wait": breakdown.get("agree_barrier_wait_ms"),
                                      "stream_drain_wait": breakdown.get("stream_drain_wait_ms")}
        t_sched = head_bytes_per_link / ((link_gbps or SURVEY_LINK_GBS) * 1e9)
        kf = _fraction(t_sched, kern_ms * 1e-3) if kern_ms > 0 and not rehearsal else {"frac": None}
        out["frac_kernels_only"] = kf["frac"]
    return out


def rd_roofline_block(world, S, t_rd, transport, link_gbps, t_direct=None, rehearsal=False, breakdown=None):
    """configs[2]: fault-tolerant recursive doubling, S bytes per rank, against link rooflines.

    The reference moves one whole buffer per step over ONE partner link (MPI_Sendrecv of the
    full vector, /root/reference/src/rd/recursive_doubling.c:21-37): L = log2(p') steps, plus
    the pre-step (reduce_pow2, rd/util.c:3-34: an extra rank sends its vector) and the fan-out
    to the extra ranks (recursive_doubling.c:78-89) when p is not a power of two -- so
    (L + 2 [rem > 0]) S per rank and direction, one link at a time.  That is also the build's
    `direct` transport.  The 2-hop relay stripes each step over r - 1 links (r = p' receivers)
    and moves 2 S / r over each (two phases), so its bound is (2 L / r) S per link (+ the
    direct pre / post steps).  Every fraction is a bound over the time of the schedule it
    bounds (`_fraction`: never above 1); `reference_schedule_frac` prices the reference's
    movement against the direct transport's own time (the same data movement, timed in the
    same job by the RD transport selection)."""
    L = world.bit_length() - 1
    r = 1 << L
    rem = world - r
    ref_bytes = (L + (2 if rem else 0)) * float(S)
    if transport == "relay2hop":
        per_link = L * 2.0 / r * S + (2 if rem else 0) * float(S)
        links = r - 1
    else:
        per_link, links = ref_bytes, 1
    priced = {}
    for tag, b in (("calibrated", link_gbps), ("nominal_76.8_assumed", XGMI_LINK_GBS),
                   ("survey_153.6_assumed", SURVEY_LINK_GBS)):
        if not b:
            continue
        t_sched = per_link / (b * 1e9)
        t_refb = ref_bytes / (b * 1e9)
        row = {"link_GBps": round(b, 2), "schedule_t_roof_ms": round(t_sched * 1e3, 4),
               "schedule": {"frac": None, "met": None} if rehearsal else _fraction(t_sched, t_rd),
               "reference_t_roof_ms": round(t_refb * 1e3, 4),
               "speedup_vs_reference_roofline": None if rehearsal else round(t_refb / t_rd, 4)}
        if t_direct:
            row["reference_schedule"] = {"frac": None, "met": None} if rehearsal else _fraction(t_refb, t_direct)
        priced[tag] = row
    basis = "calibrated" if "calibrated" in priced else "survey_153.6_assumed"
    b = priced[basis]
    out = {"config": "configs[2]: FT recursive doubling, float32 SUM, one rank per GPU",
           "transport": transport, "schedule_bytes_per_link": per_link, "links": links,
           "reference_bytes_per_rank": ref_bytes,
           "reference_definition": f"(L + 2 [p not a power of two]) S = {ref_bytes:.0f} B per rank and direction, "
                                   "one partner link per step (rd/recursive_doubling.c:21-37)",
           "basis": basis, "frac": b["schedule"]["frac"], "ms_per_step": round(t_rd * 1e3, 4),
           "speedup_vs_reference_roofline": b["speedup_vs_reference_roofline"], "priced": priced,
           "rehearsal": rehearsal}
    if "bound_violated" in b["schedule"]:
        out["bound_violated"] = b["schedule"]["bound_violated"]
    if t_direct:
        out["direct_ms"] = round(t_direct * 1e3, 4)
        out["reference_schedule_frac"] = b["reference_schedule"]["frac"]
    if breakdown and breakdown.get("call_ms") is not None and breakdown.get("kernels_ms") is not None:
        out["non_kernel_ms"] = round(max(0.0, breakdown["call_ms"] - breakdown["kernels_ms"]), 4)
        out["kernels_ms"] = breakdown["kernels_ms"]
    return out


def multi(args):
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    cpu_mode = args.device == "cpu"
    if cpu_mode and os.environ.get("FTAR_BENCH_CPU_TEST") != "1":
        raise SystemExit("--device cpu is the bench's own CPU test (FTAR_BENCH_CPU_TEST=1), never a measurement")
    # FTAR_DEVICE pins every rank to one GPU (single-GPU rehearsal of the multi-rank path;
    # RCCL refuses two ranks on one device, so such runs use --dist-backend gloo)
    rehearsal = "FTAR_DEVICE" in os.environ or cpu_mode  # every rank on one GPU
    # this job's GPUs (LOCAL_RANK = GPU on one node), or the one GPU of a rehearsal
    devices = [int(os.environ.get("FTAR_DEVICE", "0"))] if rehearsal else list(range(world))
    dog = Watchdog(args.budget, rank)
    dog.start()
    # torch is imported while rank 0 runs the side legs (the import opens no GPU device)
    imp = threading.Thread(target=lambda: importlib.import_module("torch"), daemon=True)
    imp.start()
    cpu, c5, xgmi, side_info = side_legs(args, rank, world, devices, rehearsal)
    imp.join()
    import torch
    import torch.distributed as dist
    ftar = load_package()
    if cpu_mode:  # TEST-ONLY: the product's host C on host memory (tests/hostsim), no GPU
        ftar.use_test_library(os.path.join(ROOT, "tests", "hostsim", "_build", "libftar_hostsim.so"))
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
    else:
        dev_i = int(os.environ.get("FTAR_DEVICE", local)) % max(1, torch.cuda.device_count())
        os.environ.setdefault("FTAR_DEVICE", str(dev_i))  # the library opens the same device
        torch.cuda.set_device(dev_i)
        dev = torch.device("cuda", dev_i)
        sync = torch.cuda.synchronize
    dist.init_process_group(backend=args.dist_backend)
    dist.barrier()
    if rank == 0 and os.path.exists(leg_flag("side")):
        os.unlink(leg_flag("side"))  # every rank is past side_legs
    comm = ftar.Comm.from_env()
    comm.set_profiling(False)  # kernel events only in the profiled passes (timed_split)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.rand(args.count, device=dev, generator=g) * 2 - 1
    y = torch.empty_like(x)
    S = args.count * 4
    nccl = args.dist_backend == "nccl"
    legs = {}  # per optional leg: status and seconds

    def max_over_ranks(vals):
        t = torch.tensor(vals, dtype=torch.float64)
        if nccl:
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [v.item() for v in t.cpu()]

    def time_left():
        # the same on every rank (min over ranks of each rank's budget left)
        return -max_over_ranks([-(args.budget - (time.monotonic() - T_START))])[0]

    def timed(fn, steps=None, warmup=None):
        steps = args.steps if steps is None else steps
        warmup = args.warmup if warmup is None else warmup
        for _ in range(warmup):
            fn()
        sync()
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        step0 = kern = syncw = drain = gl = gh = pw = 0.0
        for _ in range(steps):
            fn()
            st = comm.last_stats()
            step0 += st.step0_kernel_ms
            kern += st.kernel_ms
            syncw += st.sync_wait_s
            drain += st.drain_s
            gl += st.gated_launches - st.gated_skips
            gh += st.gate_holds
            pw += st.peer_waits - st.peer_wait_skips
        sync()
        t1 = time.perf_counter()
        dist.barrier()
        t, k, kall, sw, dr, gl, gh, pw = max_over_ranks([t1 - t0, step0, kern, syncw, drain, gl, gh, pw])
        timed.link_bytes = comm.last_stats().step0_link_bytes
        # where a call's time goes (max over ranks of each part, per call)
        timed.breakdown = {"call_ms": round(t / steps * 1e3, 4), "kernels_ms": round(kall / steps, 4),
                           "dominant_kernel_ms": round(k / steps, 4), "agree_barrier_wait_ms": round(sw / steps * 1e3, 4),
                           "stream_drain_wait_ms": round(dr / steps * 1e3, 4),
                           # gated launches that ran, and those given up at a barrier that waited
                           # past FTAR_GATE_HOLD_US (max over ranks, all timed calls): a gated row
                           # mostly given up measures the hold, not the gate
                           "gated_launches": int(gl), "gate_holds": int(gh),
                           # allgathers ordered behind the peers' trees on the device (FTAR_OPT_MESH_WAIT)
                           "peer_waits": int(pw)}
        return t / steps, k / steps

    def timed_split(fn):
        """Per-call time with no kernel events in the timed region (the plain cost), then
        the dominant kernel's device time from a shorter profiled pass."""
        comm.set_profiling(False)
        t, _ = timed(fn)
        plain = timed.breakdown
        comm.set_profiling(True)
        _, k = timed(fn, max(3, args.steps // 4), 1)
        # the split of the profiled pass (kernel events on: nothing is gated there), with the
        # plain pass's call time and gate counts beside it
        timed_split.breakdown = dict(timed.breakdown, profiled=True, plain_call_ms=plain["call_ms"],
                                     plain_gated_launches=plain["gated_launches"],
                                     plain_gate_holds=plain["gate_holds"])
        return t, k

    class CallFailed(RuntimeError):
        pass

    def raben():
        rc = comm.allreduce_rabenseifner(x, y)
        if rc != 0:
            raise CallFailed(f"allreduce_rabenseifner returned {rc}")

    def rd():
        rc = comm.recursive_doubling(x, y)
        if rc != 0:
            raise CallFailed(f"recursive_doubling returned {rc}")

    def quick(fn, steps=3, warmup=1):
        return timed(fn, steps, warmup)[0]

    opts = (ftar.OPT_RELAY, ftar.OPT_OVERLAP, ftar.OPT_COPY_ENGINE, ftar.OPT_REDUNDANCY, ftar.OPT_MESH, ftar.OPT_PUSH,
            ftar.OPT_TREE_UNROLL, ftar.OPT_MESH_WAIT)
    # PUSH off, one vector per tree lane and the allgather ordered on the device unless named
    pads = (0, 0, 0, 0, 0, 0, 1, 1)
    defaults = {o: comm.get_option(o) for o in opts}
    gmax_lib = comm.get_option(ftar.OPT_GATE_MAX)  # the library's mid-size gate limit (1 MiB)

    def set_opts(vals):
        vals = tuple(vals) + pads[len(vals):]
        for o, v in zip(opts, vals):
            comm.set_option(o, v)

    # Exactness on this node's GPUs, every transport: integer-valued float32 inputs that
    # change from trial to trial (so a stale cached line or a read of the previous call's
    # window cannot pass), where every partial sum is an integer below 2^24 and hence
    # exact in any order.  Each rank regenerates every rank's input from its seed and sums
    # them itself: the expected result needs no collective.  Trials reuse the same buffers
    # (the peers' mappings of our send buffer are reused too).
    xe = torch.empty(args.count, device=dev)
    ye = torch.empty_like(xe)
    want = torch.empty_like(xe)

    def int_input(out, trial, r, n):
        ge = torch.Generator(device=dev).manual_seed(7919 * trial + r)
        out[:n].copy_(torch.randint(-1024, 1024, (n,), device=dev, generator=ge, dtype=torch.int32))

    def exact_ok(fn, trials=(1, 2), n=None):
        n = args.count if n is None else n
        bad = 0
        for t in trials:
            int_input(xe, t, rank, n)
            want[:n].zero_()
            for r in range(world):
                int_input(ye, t, r, n)
                want[:n] += ye[:n]
            ye.fill_(float("nan"))
            if fn(xe, ye, count=n) != 0 or not torch.equal(ye[:n], want[:n]):
                bad += 1
        return bad

    # Transport selection before the timed run: how the node's xGMI links behave under
    # concurrent peer reads decides between the one-hop mesh (power-of-two p without a
    # spare), the 2-hop relay and plain pairwise pulls, so a short comparison (max over
    # ranks, identical on every rank) picks one.  All three give the same bits.  A
    # candidate that fails or is not bit-exact on this node never times the headline.
    selection = None
    pow2 = world & (world - 1) == 0
    if world >= 2 and not args.no_variants:
        # (mesh, relay, push): the mesh pulls the peers' parts of each block (remote loads)
        # or, mesh_push, has every rank store its parts into the owners (remote stores) --
        # which one the fabric moves faster is measured here, not assumed
        # (mesh, relay, push, tree unroll)
        cands = {}
        g0 = gmax_lib
        if pow2 and comm.get_option(ftar.OPT_MESH):
            cands["mesh"] = (1, 1, 0, 1, g0)
            if world in (4, 8):
                # 2 / 4 vectors per lane and source in the tree kernel: more loads in flight
                # per lane when the p - 1 sources are remote (xGMI latency) -- the one-GPU A/B
                # saw HBM contention only, so the node decides
                cands["mesh_u2"] = (1, 1, 0, 2, g0)
                cands["mesh_u4"] = (1, 1, 0, 4, g0)
            cands["mesh_push"] = (1, 1, 1, 1, g0)  # remote stores in the reduce-scatter
            if world <= 8:
                cands["mesh_push2"] = (1, 1, 2, 1, g0)  # ... and in the allgather
            if world > 2:
                # the allgather after a host agree round, as before the device-side wait
                # (FTAR_OPT_MESH_WAIT=0): the node times the agree the default form leaves out
                cands["mesh_host_ag"] = (1, 1, 0, 1, g0, 0)
        if world >= 3 and comm.get_option(ftar.OPT_RELAY):
            cands["relay2hop"] = (0, 1, 0, 1, g0)
        cands["direct"] = (0, 0, 0, 1, g0)
        sel_opts = (ftar.OPT_MESH, ftar.OPT_RELAY, ftar.OPT_PUSH, ftar.OPT_TREE_UNROLL, ftar.OPT_GATE_MAX,
                    ftar.OPT_MESH_WAIT)
        cands = {k: tuple(v) + (1,) * (len(sel_opts) - len(v)) for k, v in cands.items()}
        if len(cands) > 1:
            times, inexact, failed = {}, [], {}
            for name, vals in cands.items():
                for o, v in zip(sel_opts, vals):
                    comm.set_option(o, v)
                try:
                    maybe_fail(f"select:{name}")
                    if max_over_ranks([exact_ok(comm.allreduce_rabenseifner, trials=(0,))])[0]:
                        inexact.append(name)
                        continue
                    times[name] = quick(raben, steps=5, warmup=2)
                except Exception as e:
                    failed[name] = str(e)[-200:]
            if times:
                chosen = min(times, key=times.get)
                for o, v in zip(sel_opts, cands[chosen]):
                    comm.set_option(o, v)
            else:  # every one failed: keep the defaults, exact_on_node reports it
                chosen = None
                for o in sel_opts:
                    comm.set_option(o, defaults[o] if o in defaults else gmax_lib)
            selection = {f"{k}_ms": round(t * 1e3, 4) for k, t in times.items()}
            selection.update({"chosen": chosen, "inexact": inexact, "failed": failed})

    # ---- the headline: configs[3] ----
    t_rb, k_rb = timed_split(raben)
    step0_bytes = timed.link_bytes
    breakdown = timed_split.breakdown
    relayed = comm.last_stats().relayed_steps > 0
    meshed = comm.last_stats().mesh_steps > 0
    oneshot = comm.last_stats().mesh_steps == 1  # the mesh's one-launch form (p = 2, small vectors)
    push_opt = int(comm.get_option(ftar.OPT_PUSH))
    pushed = meshed and not oneshot and push_opt != 0
    unroll = int(comm.get_option(ftar.OPT_TREE_UNROLL)) if world in (4, 8) else 1
    # the allgather after a host agree round (FTAR_OPT_MESH_WAIT=0) instead of the device wait
    host_ag = meshed and not oneshot and not pushed and comm.last_stats().peer_waits == 0
    transport = "mesh-oneshot" if oneshot else ("mesh-push2" if push_opt == 2 and world <= 8 else "mesh-push") \
        if pushed else "mesh-host-ag" if host_ag else \
        (f"mesh-u{unroll}" if unroll > 1 else "mesh") if meshed else "relay2hop" if relayed else "direct"
    keep = bool(comm.last_stats().step0_copy)  # the headline call moved the reference's step-0 copy
    chosen_opts = {o: comm.get_option(o) for o in opts}
    # the headline's gate limit; every later leg runs at the library's default unless it names
    # its own
    head_gate_max = comm.get_option(ftar.OPT_GATE_MAX)
    comm.set_option(ftar.OPT_GATE_MAX, gmax_lib)

    L = world.bit_length() - 1
    r_core = 1 << L  # ranks in the power-of-two core: the receivers of every exchange step
    # Link bytes per rank per direction.  The reference's FT Raben moves
    # (2.5 - 2^(1-L)) S: its step 0 exchanges the full vector, half of it only as
    # recovery data.  At power-of-two p no handler can use that half (they all abort
    # without a spare), so the build skips it there and moves classic Rabenseifner's
    # 2 (1 - 2^-L) S.  A relayed step moves 2/r of its window per link (two phases
    # over r-1 links); a direct step moves it over one link.
    ft_bytes = (2.5 - 2.0 ** (1 - L)) * S
    classic = 2 * (1 - 2.0 ** -L) * S
    sched_bytes = ft_bytes if keep else classic
    if oneshot:
        per_link = float(S)  # every peer's whole vector over its own link (= 2 S / p at p = 2)
    elif meshed:
        per_link = 2.0 * S / world  # one hop over p - 1 links: S/p each for RS and AG
    elif relayed:
        per_link = 2.0 / r_core * sched_bytes
    elif comm.get_option(ftar.OPT_OVERLAP) != 0:
        per_link = classic
    else:
        per_link = sched_bytes
    links = (world - 1) if meshed else (r_core - 1) if relayed else 1

    def frac(v):
        # a one-GPU rehearsal has no xGMI link in the path (every "peer" read is local
        # HBM shared by all ranks): link-roofline fractions would mix yardsticks
        return None if rehearsal or v is None else round(v, 4)

    def link_cal_from(transports):
        """SURVEY.md 8d's B_link measured in this job: the probe's plain copy over one link,
        both directions loaded (pull1_bidir), where it ran on the node; otherwise the
        direct transport's RS step 0 (one kernel per rank pulling the partner's half over
        ONE link while the partner pulls ours)."""
        dcal = transports.get("direct", {})
        probe = (xgmi or {}).get("patterns", {}).get("pull1_bidir", {})
        use_probe = bool(probe.get("ok") and probe.get("GBps_per_link")) and not rehearsal
        b = probe.get("GBps_per_link") if use_probe else dcal.get("step0_pull_GBps")
        if not b:
            return None
        return {"single_link_GBps": b, "nominal_GBps_assumed": XGMI_LINK_GBS, "survey_GBps_assumed": SURVEY_LINK_GBS,
                "frac_of_nominal": frac(b / XGMI_LINK_GBS),
                "source": "xgmi_probe pull1_bidir" if use_probe else "direct step 0",
                "rehearsal_note": "one GPU: the 'link' is the shared HBM, not a calibration" if rehearsal else None,
                "direct_step0": {"kernel": "direct transport, Raben RS step 0: pull the partner's half + reduce, "
                                           "both directions loaded", "bytes": dcal.get("step0_link_bytes"),
                                 "kernel_ms": dcal.get("step0_kernel_ms"), "pull_GBps": dcal.get("step0_pull_GBps")}}

    schedule = {
        "mesh-oneshot": "Rabenseifner, one-shot mesh: every block in its owner's reduction tree in one launch "
                        "(power-of-two p, no spare)",
        "mesh": "Rabenseifner, one-hop mesh: reduce-scatter as one tree kernel over p-1 peer pulls, allgather as "
                "one multi-source pull queued right behind it and ordered on the device (each rank publishes a flag "
                "in its HBM once its tree is released; the allgather waits for the peers' flags, no host agree in "
                "between) (power-of-two p, no spare; same reduction tree as recursive halving)",
        "mesh-host-ag": "Rabenseifner, one-hop mesh, the allgather launched after the reduce-scatter's host agree round "
                        "(FTAR_OPT_MESH_WAIT=0; power-of-two p, no spare)",
        "mesh-u2": "Rabenseifner, one-hop mesh, tree kernel with 2 vectors per lane and source (more remote loads in "
                   "flight), allgather as one multi-source pull (power-of-two p, no spare; same tree)",
        "mesh-u4": "Rabenseifner, one-hop mesh, tree kernel with 4 vectors per lane and source (more remote loads in "
                   "flight), allgather as one multi-source pull (power-of-two p, no spare; same tree)",
        "mesh-push": "Rabenseifner, one-hop mesh, push form: every rank stores its part of each block into the "
                     "owner's HBM (p-1 remote-store copies in one launch), each owner reduces its block locally in the "
                     "same tree, allgather as one multi-source pull (power-of-two p, no spare)",
        "mesh-push2": "Rabenseifner, one-hop mesh, push form in both phases: remote-store copies into the owners, the "
                      "owner's tree stores its block into every peer's workspace and its own rbuf, one local copy "
                      "of the peers' blocks to rbuf (power-of-two p <= 8, no spare)",
        "relay2hop": "Rabenseifner, step by step (recursive halving + doubling), each exchange striped over 2-hop "
                     "relays",
        "direct": "Rabenseifner, step by step (recursive halving + doubling), one pairwise pull per step",
    }[transport]

    def build_line(transports, t_ref, k_ref):
        cal = link_cal_from(transports)
        b_link = cal["single_link_GBps"] if cal and not rehearsal else None
        b_price = b_link or XGMI_LINK_GBS
        t_roof = per_link / (b_price * 1e9)
        t_survey = ft_bytes / (b_price * 1e9)  # the FT schedule on one link per step
        achieved = step0_bytes / (k_rb * 1e-3) / 1e9 if k_rb > 0 else None  # RS step-0 kernels' pulled bytes
        peak = links * b_price
        line = {
            "metric": METRIC, "value": round(world * S / t_rb / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_rb * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uniform[-1,1), HBM-resident" + (" (CPU TEST: host-sim library)" if cpu_mode else ""),
            "config": {"workload": f"configs[3]: fault-tolerant Rabenseifner Allreduce, 256 MiB float32 SUM per "
                                   f"rank, one rank per MI355X -- {schedule}",
                       "schedule": schedule, "transport": transport,
                       "step0_redundancy": "full exchange (reference)" if keep else
                       "elided (no idle rank: every handler aborts, raben/errhandler.c:207-211; with a "
                       "spare the replay reads the dead rank's step-0 half in its still-mapped IN)",
                       "count": args.count, "parallelism": f"{world} ranks"},
            "algbw_GBps": round(S / t_rb / 1e9, 2),
            "transport": transport,
            # the headline call of the profiled pass split into device time (all kernels /
            # the dominant one) and the host's waits (agree + barrier rounds, stream drains)
            "call_breakdown": breakdown,
            "north_star": north_star_block(world, S, t_rb, transport, b_link, links, per_link, t_ref, rehearsal,
                                           breakdown),
            "schedule_link_roofline": {"schedule_bytes_per_rank": sched_bytes, "bytes_per_link": per_link,
                                       "links_per_step": links,
                                       "link_GBps": b_price,
                                       "link_basis": "calibrated" if b_link else "nominal 76.8 GB/s per direction "
                                                                                 "(assumption)",
                                       "t_roof_ms": round(t_roof * 1e3, 4), "frac": frac(t_roof / t_rb),
                                       "frac_nominal_76.8": frac(per_link / (XGMI_LINK_GBS * 1e9) / t_rb),
                                       "frac_survey_153.6": frac(per_link / (SURVEY_LINK_GBS * 1e9) / t_rb)},
            "link_calibration": cal,
            "xgmi_probe": xgmi,
            "roofline": {"bound": "xgmi", "achieved": round(achieved, 1) if achieved else None,
                         "peak": round(peak, 2), "unit": "GB/s",
                         "peak_basis": f"{links} link(s) x " + (f"{b_link} GB/s calibrated" if b_link else
                                                               f"{XGMI_LINK_GBS} GB/s nominal (assumption)"),
                         "frac": frac(achieved / peak) if achieved else None,
                         "frac_nominal_76.8": frac(achieved / (links * XGMI_LINK_GBS)) if achieved else None,
                         "rehearsal": rehearsal,
                         # HBM bytes per launch from PMC exist for the one-GPU rehearsal only
                         # (every peer on this device); on the node the peer reads hit the
                         # peers' HBM and the counters of one device miss them
                         "traffic": pmc_traffic(f"mesh_tree_p{world}_rehearsal")[0] if rehearsal and meshed
                         and not oneshot else None,
                         "traffic_source": pmc_traffic(f"mesh_tree_p{world}_rehearsal")[1] if rehearsal and meshed
                         and not oneshot else None,
                         "traffic_note": "PMC counters of a peer-reading kernel are per device; not collected on "
                                         "the 8-GPU node (profiles/pmc_summary.json has the one-GPU rehearsal's: "
                                         "tree and allgather kernels within 0.02 % of their algorithmic bytes)",
                         "kernel": ("Raben one-shot mesh: tree_batch_kernel, every block in its owner's tree"
                                    if oneshot
                                    else "Raben mesh reduce-scatter, push form: p-1 remote-store copies in one launch"
                                    if pushed
                                    else "Raben mesh reduce-scatter: tree_kernel over p-1 one-hop pulls" if meshed
                                    else "Raben RS step 0, both relay phases (stripes pulled over r-1 links)" if relayed
                                    else "Raben RS step 0 reduce half (pull partner's half, reduce into W)"),
                         "algorithmic_bytes_per_launch": step0_bytes, "kernel_ms": round(k_rb, 4)},
            "transport_selection": selection,
            "cpu_baseline": cpu,
            "side_legs": side_info,
        }
        if t_ref:
            line["reference_shape"] = {
                "schedule": "Rabenseifner step by step, pairwise pulls (one xGMI link per step), step-0 full-vector "
                            "exchange kept (raben/rabenseifner.c:206-211)",
                "value": round(world * S / t_ref / 1e9, 2), "ms_per_step": round(t_ref * 1e3, 4),
                "algbw_GBps": round(S / t_ref / 1e9, 2), "step0_kernel_ms": round(k_ref, 4),
                "survey_ft_roofline_ms": round(t_survey * 1e3, 4),
                "frac_of_survey_roofline": frac(t_survey / t_ref),
                "frac_of_survey_roofline_nominal_76.8": frac(ft_bytes / (XGMI_LINK_GBS * 1e9) / t_ref),
                "frac_of_survey_roofline_survey_153.6": frac(ft_bytes / (SURVEY_LINK_GBS * 1e9) / t_ref)}
        return line

    line = build_line({}, None, 0.0)
    dog.line = line
    if rank == 0:
        print(json.dumps(dict(line, line="headline")), flush=True)

    # ---- optional legs: each runs only while the budget has room, records its own fate ----
    def opt_leg(name, est_s, fn):
        t0 = time.monotonic()
        if time_left() < est_s:
            legs[name] = {"status": "skipped", "reason": f"budget: needs ~{est_s:.0f} s"}
            return None
        try:
            maybe_fail(name)
            if test_hook("hang", name):  # TEST-ONLY: an in-process leg that never returns
                time.sleep(3600)
            r = fn()
            legs[name] = {"status": "ok", "s": round(time.monotonic() - t0, 2)}
            return r
        except Exception as e:  # uniform on every rank for the failures a leg raises itself
            legs[name] = {"status": "error", "s": round(time.monotonic() - t0, 2), "error": str(e)[-400:]}
            return None

    def checks_leg():
        # correctness spot check against torch.distributed's all_reduce on the same inputs
        # (fp32, different reduction order: |err| <= log2(p) * 2^-24 * sum|x_i|)
        ref = x.clone() if nccl or cpu_mode else x.cpu()
        dist.all_reduce(ref)
        raben()
        err = (y.cpu() - ref.cpu()).abs().max().item()
        # the reference drivers' case (buffer[i] = rank, int32 SUM): closed-form checksum
        # sum_i result[i] % 17 = ((p (p-1) / 2) % 17) * count  (analysis/check_fault.py:62-67)
        xi = torch.full((args.count,), rank, dtype=torch.int32, device=dev)
        yi = torch.empty_like(xi)
        if comm.allreduce_rabenseifner(xi, yi) != 0:
            raise CallFailed("int32 Rabenseifner failed")
        cks_raben = int((yi.to(torch.int64) % 17).sum().item())
        if comm.recursive_doubling(xi, yi) != 0:
            raise CallFailed("int32 recursive doubling failed")
        cks_rd = int((yi.to(torch.int64) % 17).sum().item())
        cks_want = ((world * (world - 1) // 2) % 17) * args.count
        return err, {"raben": cks_raben == cks_want, "rd": cks_rd == cks_want}

    # The small-call mechanisms -- completion signalled by the kernels themselves
    # (<= 64 workgroups), inputs staged below FTAR_STAGE_MAX, launches queued behind gates
    # (Raben one-shot below FTAR_ONESHOT_MAX, RD steps) -- each has a size threshold near
    # 1 MiB; the checks straddle it, gated and ungated, for both schedules.
    EXACT_SIZES = (("4B", 1), ("4KiB", 1024), ("64KiB", 16384), ("1MiB-16B", 262140), ("1MiB", 262144),
                   ("1MiB+16B", 262148), ("4MiB", 1 << 20))
    MID_GATE_MAX = 16 << 20  # the mid-size gates' range the size sweep times (FTAR_OPT_GATE_MAX)
    small_fallback = {}

    def exact_leg():
        # Exactness of every transport and mechanism on this node (helpers above the selection)
        base = [chosen_opts[o] for o in opts]
        raben_fn, rd_fn = comm.allreduce_rabenseifner, comm.recursive_doubling
        # (name, option values, function, count or None = the job's, extra options)
        checks = [("chosen", base, raben_fn, None, {ftar.OPT_GATE_MAX: head_gate_max}),
                  ("reference_shape", (0, 0, 0, 1, 0), raben_fn, None, {}),
                  ("rd", base, rd_fn, None, {}),
                  ("chosen_64KiB", base, raben_fn, 16384, {})]
        small = []  # the checks of the small-call mechanisms (the fallback below reruns them)
        for label, n in EXACT_SIZES:
            if n > args.count:
                continue
            for algo, fn in (("raben", raben_fn), ("rd", rd_fn)):
                for gate in (1, 0):
                    more = {ftar.OPT_GATE: gate}
                    if gate and 4 * n > (1 << 20):  # mid-size: the relayed gates (off by default)
                        more[ftar.OPT_GATE_MAX] = MID_GATE_MAX
                    small.append((f"{algo}_{label}_{'gated' if gate else 'ungated'}", base, fn, n, more))
        checks += small
        if not args.no_variants:
            checks += [(name, vals, raben_fn, None, {}) for name, vals in
                       (("mesh", (1, 1, 0, 0, 1)), ("mesh_u2", (1, 1, 0, 0, 1, 0, 2)), ("mesh_u4", (1, 1, 0, 0, 1, 0, 4)),
                        ("mesh_push", (1, 1, 0, 0, 1, 1)), ("mesh_push2", (1, 1, 0, 0, 1, 2)),
                        ("relay2hop", (1, 1, 0, 0, 0)), ("direct", (0, 1, 0, 0, 0)), ("copy_engine", (0, 1, 1, 0, 0)))
                       if pow2 or not name.startswith("mesh")]
            if pow2 and world > 2:
                # the allgather after the reduce-scatter's host agree (transport selection's mesh_host_ag)
                checks.append(("mesh_host_ag", (1, 1, 0, 0, 1, 0, 1, 0), raben_fn, None, {}))
            if pow2:
                checks += [(name, vals, raben_fn, min(16384, args.count), {}) for name, vals in
                           (("mesh_push_64KiB", (1, 1, 0, 0, 1, 1)), ("mesh_push2_64KiB", (1, 1, 0, 0, 1, 2)),
                            ("mesh_u4_64KiB", (1, 1, 0, 0, 1, 0, 4)))]
            checks += [("rd_relay", (1, 1, 0, 0, 0), rd_fn, None, {}),
                       ("rd_direct", (0, 1, 0, 0, 0), rd_fn, None, {})]
        gate0 = comm.get_option(ftar.OPT_GATE)
        gmax0 = comm.get_option(ftar.OPT_GATE_MAX)
        flag0 = comm.get_option(ftar.OPT_FLAG_SYNC)

        def run(cks, extra=None):
            fails = []
            for name, vals, fn, n, more in cks:
                set_opts(vals)
                if name == "rd" and rd_selection:  # the transport the RD timing chose
                    comm.set_option(ftar.OPT_RELAY, int(rd_selection["chosen"] == "relay2hop"))
                for o, v in {**more, **(extra or {})}.items():
                    comm.set_option(o, v)
                maybe_fail(f"exact:{name}")
                fails.append(exact_ok(fn, n=n))
                comm.set_option(ftar.OPT_GATE, gate0)
                comm.set_option(ftar.OPT_GATE_MAX, gmax0)
            return max_over_ranks(fails) if fails else []

        comm.set_profiling(False)
        try:
            fails = run(checks)
            exact = {"inputs": "integer-valued float32 in [-1024, 1024), new per trial, 2 trials per check; "
                               "expected sum regenerated on every rank (exact in any order)",
                     "all_exact": all(f == 0 for f in fails)}
            exact.update({name: f == 0 for (name, _, _, _, _), f in zip(checks, fails)})
            # A small-call check that is not exact says which mechanism broke: rerun the failing
            # ones with the gates off, then also with the kernels' completion flags off (fenced
            # marker drains), and keep the first setting under which all of them are exact for
            # the rest of the job -- the size sweep is timed with it.
            bad = [c for c, f in zip(checks, fails) if f]
            if any(c in small for c in bad):
                tried = []
                chosen_setting = None
                for label, extra in (("gate=0", {ftar.OPT_GATE: 0}),
                                     ("gate=0,flag_sync=0", {ftar.OPT_GATE: 0, ftar.OPT_FLAG_SYNC: 0})):
                    f2 = run(bad, extra)  # every failing check (a small mesh call is gated too)
                    comm.set_option(ftar.OPT_FLAG_SYNC, flag0)
                    still = [c[0] for c, f in zip(bad, f2) if f]
                    tried.append({"setting": label, "exact": not still, "still_inexact": still})
                    if not any(c in small for c, f in zip(bad, f2) if f):
                        chosen_setting = (label, extra, not still)
                        break
                small_fallback.update({"failed": [c[0] for c in bad], "tried": tried,
                                       "setting": chosen_setting[0] if chosen_setting else None})
                if chosen_setting:
                    for o, v in chosen_setting[1].items():
                        comm.set_option(o, v)
                exact["small_call_fallback"] = small_fallback
                exact["all_exact_after_fallback"] = bool(chosen_setting and chosen_setting[2])
        finally:
            set_opts([chosen_opts[o] for o in opts])
            comm.set_profiling(True)
        return exact

    def ref_shape_leg():
        # The reference's own data movement, first class: pairwise pulls, step by step, one
        # link per step, with the step-0 full-vector exchange kept (its tmp redundancy,
        # raben/rabenseifner.c:206-211) even where no handler can use it.
        set_opts((0, 0, 0, 1, 0))
        try:
            return timed_split(raben)
        finally:
            set_opts([chosen_opts[o] for o in opts])

    rd_selection = None
    rd_raw = {}

    def rd_leg():
        # recursive doubling has no mesh form (it can recover at any p): relay or direct
        nonlocal rd_selection
        relay_for_raben = comm.get_option(ftar.OPT_RELAY)
        try:
            if world >= 3 and not args.no_variants:
                comm.set_option(ftar.OPT_RELAY, 1)
                t_r = quick(rd)
                comm.set_option(ftar.OPT_RELAY, 0)
                t_d = quick(rd)
                comm.set_option(ftar.OPT_RELAY, 1 if t_r <= t_d else 0)
                rd_selection = {"relay2hop_ms": round(t_r * 1e3, 4), "direct_ms": round(t_d * 1e3, 4),
                                "chosen": "relay2hop" if t_r <= t_d else "direct"}
            t_rd, k_rd = timed_split(rd)
            rd_raw.update(t=t_rd, breakdown=timed_split.breakdown,
                          transport="relay2hop" if comm.last_stats().relayed_steps > 0 else "direct",
                          t_direct=t_d if rd_selection else (t_rd if world == 2 else None))
        finally:
            comm.set_option(ftar.OPT_RELAY, relay_for_raben)
        return {"ms_per_step": round(t_rd * 1e3, 4), "algbw_GBps": round(S / t_rd / 1e9, 2),
                "value": round(world * S / t_rd / 1e9, 2), "step0_kernel_ms": round(k_rd, 4),
                "transport": rd_raw["transport"], "call_breakdown": timed_split.breakdown,
                "transport_selection": rd_selection}

    def rccl_leg():
        zz = x.clone()
        t_nc, _ = timed(lambda: dist.all_reduce(zz))
        return {"ms_per_step": round(t_nc * 1e3, 4), "algbw_GBps": round(S / t_nc / 1e9, 2),
                "value": round(world * S / t_nc / 1e9, 2)}

    def transports_leg():
        # mesh: one-hop reduce-scatter + allgather (power-of-two p, no spare); relay2hop:
        # the step-by-step schedule striped over 2-hop paths; direct: one pull kernel per
        # step; direct_serial: plus the step-0 copy inline; copy_engine: hipMemcpyAsync of
        # the partner's window + a local reduce kernel; relay_full_exchange: the relay with
        # the reference's step-0 full exchange.  Each variant records its own failure.
        out = {}
        variants = (("mesh", (1, 1, 0, 0, 1)), ("mesh_host_ag", (1, 1, 0, 0, 1, 0, 1, 0)),
                    ("mesh_push", (1, 1, 0, 0, 1, 1)), ("mesh_push2", (1, 1, 0, 0, 1, 2)),
                    ("relay2hop", (1, 1, 0, 0, 0)),
                    ("direct", (0, 1, 0, 0, 0)), ("direct_serial", (0, 0, 0, 0, 0)), ("copy_engine", (0, 1, 1, 0, 0)),
                    ("relay_full_exchange", (1, 1, 0, 1, 0)))
        try:
            for name, vals in variants:
                if name.startswith("mesh") and not pow2:
                    continue
                if time_left() < 10:
                    out[name] = {"skipped": "budget"}
                    continue
                if name == "mesh_host_ag" and world == 2:
                    continue
                try:
                    maybe_fail(f"transports:{name}")
                    set_opts(vals)
                    comm.set_option(ftar.OPT_GATE_MAX, gmax_lib)  # every variant at the library's gate limit
                    tv, kv = timed_split(raben)
                    lb = timed.link_bytes
                    tv_rd = timed(rd)[0] if name in ("relay2hop", "direct", "copy_engine") else None
                    bd = timed_split.breakdown
                    out[name] = {"raben_ms": round(tv * 1e3, 4), "raben_algbw_GBps": round(S / tv / 1e9, 2),
                                 "step0_kernel_ms": round(kv, 4), "step0_link_bytes": lb,
                                 "step0_pull_GBps": round(lb / (kv * 1e-3) / 1e9, 2) if kv > 0 else None,
                                 # the call's time outside its kernels (plain call - profiled kernels)
                                 "kernels_ms": bd.get("kernels_ms"),
                                 "non_kernel_ms": round(bd["plain_call_ms"] - bd["kernels_ms"], 4)
                                 if bd.get("plain_call_ms") is not None and bd.get("kernels_ms") is not None else None,
                                 "agree_barrier_wait_ms": bd.get("agree_barrier_wait_ms"),
                                 "peer_waits": bd.get("peer_waits")}
                    if tv_rd:
                        out[name].update({"rd_ms": round(tv_rd * 1e3, 4), "rd_algbw_GBps": round(S / tv_rd / 1e9, 2)})
                except Exception as e:
                    out[name] = {"error": str(e)[-300:]}
        finally:
            set_opts([chosen_opts[o] for o in opts])
            comm.set_option(ftar.OPT_GATE_MAX, gmax_lib)
        return out

    def sweep_leg():
        # Per-call time over message sizes (max over ranks), 4 B .. 512 MiB, with the chosen
        # transport, next to RCCL's all_reduce on the same sizes: the FT/vendor curve of the
        # reference's compare campaign (slurm/test_compare.slurm:27-50, check_compare.py),
        # plus the fixed cost per call and the one-shot threshold (FTAR_ONESHOT_MAX)
        # timed with the small-call setting exact_on_node kept (a fallback if a gated or
        # flag-signalled check was not exact on this node)
        sizes = {"small_call_setting": small_fallback.get("setting") or "default (gates, flag-signalled drains)",
                 "gate": comm.get_option(ftar.OPT_GATE), "flag_sync": comm.get_option(ftar.OPT_FLAG_SYNC)}
        comm.set_profiling(False)  # no kernel events: the plain per-call cost
        oneshot_max = comm.get_option(ftar.OPT_ONESHOT_MAX)
        gate_max0 = comm.get_option(ftar.OPT_GATE_MAX)
        z = x.clone() if nccl else None
        n = 1
        try:
            while n <= args.count:
                if time_left() < 15:
                    sizes["truncated_at_bytes"] = 4 * n
                    break
                # small calls: a long warm-up, so the timed calls see a GPU and host cores that
                # are past their idle power states (a cold start measured 2-3x the per-call
                # time in one-GPU rehearsals, profiles/r03/README.md)
                steps, warm = (100, 50) if 4 * n <= (1 << 20) else (20, 3) if n <= (1 << 22) else (5, 2)
                row = {"bytes": 4 * n}
                mid = gate_max0 < 4 * n <= MID_GATE_MAX and comm.get_option(ftar.OPT_GATE) != 0
                for name, fn, extra in (("raben", comm.allreduce_rabenseifner, None),
                                        ("raben_no_oneshot", comm.allreduce_rabenseifner, {ftar.OPT_ONESHOT_MAX: 0}),
                                        ("rd", comm.recursive_doubling, None),
                                        # mid-size RD calls with steps 1.. queued behind relayed
                                        # gates (off by default: DESIGN.md 6; the mesh's allgather
                                        # is ordered on the device instead)
                                        ("rd_midgate", comm.recursive_doubling, {ftar.OPT_GATE_MAX: MID_GATE_MAX})):
                    if name == "raben_no_oneshot" and (not (pow2 and comm.get_option(ftar.OPT_MESH) and oneshot_max > 0)
                                                       or (world > 2 and 4 * n > oneshot_max)):
                        continue
                    if name.endswith("_midgate") and not mid:
                        continue
                    for o, v in (extra or {}).items():
                        comm.set_option(o, v)

                    def call(fn=fn, n=n):
                        if fn(x, y, count=n) != 0:
                            raise CallFailed(f"size sweep call of {4 * n} B failed")

                    try:
                        row[name + "_us"] = round(quick(call, steps=steps, warmup=warm) * 1e6, 2)
                        if 4 * n in (4, 65536):  # where a small call's time goes (max over ranks)
                            row[name + "_split_us"] = {
                                "drain": round(timed.breakdown["stream_drain_wait_ms"] * 1e3, 2),
                                "agree_barrier": round(timed.breakdown["agree_barrier_wait_ms"] * 1e3, 2),
                                "gated_launches": timed.breakdown["gated_launches"],
                                "gate_holds": timed.breakdown["gate_holds"]}
                        if name.endswith("_midgate") or timed.breakdown["gate_holds"]:
                            row[name + "_gate_holds"] = timed.breakdown["gate_holds"]
                    finally:
                        comm.set_option(ftar.OPT_ONESHOT_MAX, oneshot_max)
                        comm.set_option(ftar.OPT_GATE_MAX, gate_max0)
                if z is not None:
                    zn = z[:n]
                    row["rccl_us"] = round(quick(lambda: dist.all_reduce(zn), steps=steps, warmup=warm) * 1e6, 2)
                    row["raben_over_rccl"] = round(row["raben_us"] / row["rccl_us"], 3)
                sizes[str(4 * n)] = row
                n *= 2
            if n == 2 * args.count and "truncated_at_bytes" not in sizes:
                # the reference's campaign ends at 2^27 ints = 512 MiB (run/run_compare.sh): one
                # more point on a vector twice the job's, allocated for it and freed after
                if time_left() < 20:
                    sizes["truncated_at_bytes"] = 4 * n
                else:
                    xb = torch.cat([x, x])
                    yb = torch.empty_like(xb)
                    row = {"bytes": 4 * n}
                    for name, fn in (("raben", comm.allreduce_rabenseifner), ("rd", comm.recursive_doubling)):
                        def call(fn=fn):
                            if fn(xb, yb) != 0:
                                raise CallFailed(f"size sweep call of {4 * n} B failed")

                        row[name + "_us"] = round(quick(call, steps=5, warmup=2) * 1e6, 2)
                    if z is not None:
                        row["rccl_us"] = round(quick(lambda: dist.all_reduce(xb), steps=5, warmup=2) * 1e6, 2)
                        row["raben_over_rccl"] = round(row["raben_us"] / row["rccl_us"], 3)
                    sizes[str(4 * n)] = row
                    del xb, yb
        finally:
            comm.set_profiling(True)
        return sizes

    def e2e_leg():
        # end-to-end with host buffers: pinned H2D + device Allreduce + D2H (never the value)
        xh = x.cpu() if cpu_mode else x.cpu().pin_memory()
        yh = torch.empty_like(xh) if cpu_mode else torch.empty_like(xh).pin_memory()

        def raben_host():
            if comm.allreduce_rabenseifner_host(xh, yh) != 0:
                raise CallFailed("host-buffer Rabenseifner failed")

        t_e2e, _ = timed(raben_host, 3, 1)
        return {"ms_per_step": round(t_e2e * 1e3, 3), "algbw_GBps": round(S / t_e2e / 1e9, 2)}

    final = {}
    ck = opt_leg("checks", 10, checks_leg)
    if ck:
        final["max_abs_err_vs_rccl"], final["int32_rank_checksum_ok"] = ck
    rs = opt_leg("reference_shape", 15, ref_shape_leg)
    t_ref, k_ref = rs if rs else (None, 0.0)
    final["rd"] = opt_leg("rd", 15, rd_leg)
    final["exact_on_node"] = opt_leg("exact_on_node", 30, exact_leg)
    final["rccl_allreduce"] = opt_leg("rccl_allreduce", 10, rccl_leg) if nccl else None
    transports = {} if args.no_variants else (opt_leg("transports", 40, transports_leg) or {})
    final["transports"] = transports
    final["size_sweep_us"] = {} if args.no_variants else opt_leg("size_sweep", 40, sweep_leg)
    final["e2e_host_buffers"] = opt_leg("e2e_host_buffers", 20, e2e_leg)
    del xe, ye, want

    # IPC exports the runtime refused and the library re-allocated (expected 0)
    final["export_retries_max_over_ranks"] = int(max_over_ranks([float(comm.last_stats().export_retries)])[0])
    # calls that found the caller's stream busy and waited for it on the host
    final["user_stream_waits_max_over_ranks"] = int(max_over_ranks([float(comm.last_stats().user_stream_waits)])[0])
    line = build_line(transports, t_ref, k_ref)
    if final.get("rd") and rd_raw.get("t"):
        # configs[2] against its link rooflines, priced at the same link as the headline
        cal = link_cal_from(transports)
        final["rd"]["schedule_link_roofline"] = rd_roofline_block(
            world, S, rd_raw["t"], rd_raw["transport"], cal["single_link_GBps"] if cal and not rehearsal else None,
            rd_raw.get("t_direct"), rehearsal, rd_raw.get("breakdown"))
    line.update(final)
    line["c5_single_kill"] = c5
    line["legs"] = legs
    line["job_s"] = round(time.monotonic() - T_START, 1)
    try:  # what this run decides for the next build (analysis/analyze.py decisions)
        line["node_decisions"] = load_analysis().decisions(line)
    except Exception as e:  # a summary, never the line's fate
        line["node_decisions"] = {"error": str(e)[-200:]}
    dog.line = line
    if rank == 0:
        print(json.dumps(dict(line, line="final")), flush=True)
    dog.done.set()
    comm.finalize()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--count", type=int, default=COUNT)
    ap.add_argument("--pairs", type=int, default=4, help="N=1: rotating vector pairs (4 x 2 x 256 MiB = 2 GiB)")
    ap.add_argument("--variant", type=int, default=1, help="local-reduce kernel: 0 register, 1 LDS-DMA (default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="N>1: skip the configs[4] single-kill leg")
    ap.add_argument("--no-xgmi", action="store_true", help="N>1: skip the xGMI fabric probe")
    ap.add_argument("--timing", choices=["region", "launch"], default="region",
                    help="N=1 kernel time: events around the timed region, or around every launch")
    ap.add_argument("--no-variants", action="store_true", help="N>1: skip the transport comparison and size sweep")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for barrier/timing")
    ap.add_argument("--side-budget", type=float, default=150.0,
                    help="N>1: seconds for all side legs together (CPU baseline, fabric probe, configs[4] jobs)")
    ap.add_argument("--budget", type=float, default=480.0,
                    help="N>1: seconds for the whole job; optional legs run only while it has room")
    ap.add_argument("--c5-draws", type=int, default=10, help="N>1: random-kill draws of the configs[4] campaign")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu", help=argparse.SUPPRESS)
    ap.add_argument("--no-pmc", action="store_true", help="N=1: skip the live rocprofv3 --pmc traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.pmc_child:
        args.steps = args.steps or 20
        return pmc_child(args)
    if world > 1:
        args.steps = args.steps or 20
        args.warmup = args.warmup if args.warmup is not None else 3
        multi(args)
    else:
        args.steps = args.steps or 200
        args.warmup = args.warmup if args.warmup is not None else 10
        single(args)


if __name__ == "__main__":
    main()
