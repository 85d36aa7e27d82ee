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
       GPUs + one idle spare, a kill mid-exchange, recovery) are reported beside it.

value = (input vectors summed x bytes per vector) / time per step, whole job:
        N=1: 2 x 256 MiB per launch; N>1: N x 256 MiB per Allreduce.
Data are synthetic (uniform [-1, 1)), inputs resident in HBM before timing starts.
"""
import argparse
import importlib.util
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
COUNT = 1 << 26              # 256 MiB of float32 per vector
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 76.8         # one xGMI link, one direction (153.6 GB/s bidirectional spec)
METRIC = "Allreduce GB/s (device-resident, float32 SUM) at 1/2/4/8 MI355X"
# data/data_fault/log_single_Raben.csv, N = 9, OK runs: median clock() seconds
REF_C5_S = {"kill": 1.334, "no_kill": 1.329, "count": 120732254}


def load_package():
    path = os.path.join(ROOT, "fault-tolerant_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("ftar_amd", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ftar_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pmc_traffic(name):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(name, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


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


def cpu_schedule(algo, p, count, reps):
    """The schedule on the host cores: the product's host C (control plane, agree rounds,
    the FT schedule) as p processes pinned one per core, POSIX shared memory as the
    transport, C loops as the reduce (tools/cpu_schedule_bench.py), float32."""
    cs = load_tool("cpu_schedule_bench")
    cs.build()
    r = cs.run(algo, p, count, "float32", reps)
    return r, cs.cpu_model()


def c1_baseline():
    """BASELINE configs[0]: src/rd/main recursive doubling, float32 SUM, 64 KiB, 4 ranks."""
    r, model = cpu_schedule("rd", 4, 16384, 20)
    return {"value": round(4 * 16384 * 4 / r["time_s"] / 1e9, 4), "unit": "GB/s", "ms_per_call": round(r["time_s"] * 1e3, 4),
            "algbw_GBps": r["algbw_GBps"], "cores": 4, "kind": "port", "cpu_model": model,
            "sample": "configs[0]: recursive doubling, 64 KiB float32 SUM per rank, 4 rank processes pinned one "
                      "per core, pairwise step-by-step exchanges through shared memory, median of 20 runs "
                      "(value = 4 x 64 KiB / call time, as the GPU lines)",
            "reference_leonardo_ms": 0.976}


def single(args):
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
                     "traffic": pmc_traffic("reduce_local_c2_lds_rot" if args.variant == 1 else "reduce_local_c2_rot"),
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


def c5_leg(world, devices, count, ranks, calls=6, kill_call=2):
    """configs[4] on this node: `ranks` = world GPUs' worth of ranks + one idle spare (rank
    1 shares rank 0's GPU), Rabenseifner 256 MiB float32 SUM, `calls` calls per job; the
    fault job kills vrank 5 (original rank 6) in reduce-scatter step 1 of call `kill_call`,
    mid-exchange (its own pull kernel in flight, its partner's pull reading its HBM), a
    second one in allgather step 1 ("also AG step 1"; the last AG step when
    there are only two).  The recovery shrinks the comm; the later calls run on the
    survivors.  Call 0 is the warm-up (workspace allocation, IPC imports).  Run by rank 0
    as separate ftrun jobs of bin/ftbench: torchrun's agent would tear the job down on a
    SIGKILL."""
    exe = os.path.join(ROOT, "fault-tolerant_amd", "bin", "ftbench")
    ftrun = os.path.join(ROOT, "fault-tolerant_amd", "bin", "ftrun")
    devmap = [devices[0], devices[0]] + [devices[(r - 1) % len(devices)] for r in range(2, ranks)]
    victim = 6 if ranks > 6 else ranks - 1
    ag_step = 1 if ranks >= 8 else 0  # a middle allgather step where there is one (L >= 3)
    env = {k: v for k, v in os.environ.items()
           if not k.startswith(("FTAR_", "RANK", "LOCAL_", "WORLD_", "GROUP_", "ROLE_", "TORCHELASTIC"))}
    res = {"ranks": ranks, "devmap": devmap, "count": count, "calls": calls,
           "kill": f"{victim}:1:1:3 in call {kill_call} (original rank {victim} = vrank {victim - 1}, reduce-scatter "
                   "step 1, mid-exchange)",
           "kill_ag": f"{victim}:2:{ag_step}:3 in call {kill_call} (allgather step {ag_step}, mid-exchange)"}
    want_all = float(sum(range(ranks)))
    for name, kill in (("no_fault", None), ("fault", f"{victim}:1:1:3:{kill_call}"),
                       ("fault_ag", f"{victim}:2:{ag_step}:3:{kill_call}")):
        e = dict(env)
        if kill:
            e["FTAR_KILL"] = kill
        t0 = time.time()
        cp = subprocess.run([ftrun, "-np", str(ranks), "--devmap", ",".join(map(str, devmap)), exe, "raben",
                             str(count), str(calls)], env=e, capture_output=True, text=True, timeout=180)
        lines = [json.loads(l) for l in cp.stdout.splitlines() if l.startswith("{")]
        per_call = []
        for c in range(calls):
            per = [ln["calls"][c] for ln in lines]
            # the kill call still sums every input (the dead rank's block is recovered,
            # the reference's corr path); later calls sum the survivors'
            want = want_all - (victim if (kill and c > kill_call) else 0)
            per_call.append({"ms_max_over_ranks": round(max(p["ms"] for p in per), 3) if per else None,
                             "recoveries": max((p["recoveries"] for p in per), default=None),
                             "comm_size_after": min((p["comm_size"] for p in per), default=None),
                             "result_ok": bool(per) and all(p["rc"] == 0 and p["uniform"] and p["value"] == want
                                                            for p in per)})
        res[name] = {"rc": cp.returncode, "survivors": len(lines), "job_wall_s": round(time.time() - t0, 2),
                     "calls": per_call}
        if cp.returncode != 0 or not lines:
            res[name]["stderr_tail"] = cp.stderr[-600:]
        mid = [l for l in cp.stderr.splitlines() if "dies mid-exchange" in l]
        if mid:
            res[name]["victim"] = mid[0].split("ftar: ")[-1]
    res["random_kill"] = c5_random_kill(ftrun, exe, ranks, devmap, count, env)
    f, n = res.get("fault", {}), res.get("no_fault", {})

    def med(cs):
        v = sorted(c["ms_max_over_ranks"] for c in cs)
        return v[len(v) // 2]
    def recovered(job):
        fc = job["calls"]
        return job["survivors"] == ranks - 1 and fc[kill_call]["recoveries"] == 1 and all(c["result_ok"] for c in fc)
    try:
        fc = f["calls"]
        res["recovered_rs"] = recovered(f)
        res["recovered_ag"] = recovered(res["fault_ag"])
        res["recovered"] = res["recovered_rs"] and res["recovered_ag"]
        res["recovered_call_ms"] = fc[kill_call]["ms_max_over_ranks"]
        res["recovered_ag_call_ms"] = res["fault_ag"]["calls"][kill_call]["ms_max_over_ranks"]
        res["no_fault_call_ms"] = med(n["calls"][1:])  # median after the warm-up call
        res["recovery_overhead_ms"] = round(res["recovered_call_ms"] - res["no_fault_call_ms"], 3)
        res["pre_fault_call_ms"] = med(fc[1:kill_call])
        res["survivors_call_ms"] = med(fc[kill_call + 1:])  # p - 1 ranks after the shrink
    except (KeyError, IndexError, TypeError, ValueError):
        res["recovered"] = False
    res["reference_leonardo_s"] = dict(REF_C5_S, note="clock() s per run incl. the whole MPI job, 460.6 MiB int32")
    return res


def c5_random_kill(ftrun, exe, ranks, devmap, count, env, calls=3, loop_s=1.5, seed=0):
    """The reference's random kill (run/kill_procs.sh: SIGKILL one rank process after a
    random delay) on the configs[4] job: each call is stretched to `loop_s` seconds of
    busy agree rounds (FTAR_LOOP_SECONDS, as run/run_mpi.sh does) so the kill lands inside
    the schedule; the outcome is the reference's (recovered, or MPI_Abort where its
    handler aborts), and every survivor's results must agree, call by call, on the exact
    sum with or without the victim's input, never dropping it and taking it back."""
    import random
    import signal
    rng = random.Random(seed)
    victim = rng.randrange(ranks)
    delay = rng.uniform(1.0, 1.0 + loop_s * calls)  # after the launch: ~1 s of process start-up
    e = dict(env, FTAR_LOOP_SECONDS=str(loop_s))
    out = {"victim": victim, "delay_s": round(delay, 3), "loop_seconds": loop_s, "calls": calls}
    pr = None
    try:
        import psutil
        t0 = time.time()
        pr = subprocess.Popen([ftrun, "-np", str(ranks), "--devmap", ",".join(map(str, devmap)), exe, "raben",
                               str(count), str(calls)], env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        time.sleep(delay)
        for k in psutil.Process(pr.pid).children():  # the rank processes ftrun started
            try:
                if k.environ().get("FTAR_RANK") == str(victim):
                    os.kill(k.pid, signal.SIGKILL)
                    out["killed"] = True
            except (psutil.Error, OSError):
                pass
        so, se = pr.communicate(timeout=180)
        out["job_wall_s"] = round(time.time() - t0, 2)
    except Exception as ex:
        out["error"] = str(ex)[-300:]
        if pr is not None and pr.poll() is None:
            pr.kill()  # ftrun's ranks follow it (PR_SET_PDEATHSIG)
            pr.wait()
        return out
    lines = [json.loads(l) for l in so.splitlines() if l.startswith("{")]
    full = float(sum(range(ranks)))
    out["aborted"] = "MPI_ABORT" in se
    out["survivors"] = len(lines)
    consistent = bool(lines) or out["aborted"]
    dropped = False
    per = []
    for c in range(calls):
        vals = {ln["calls"][c]["value"] for ln in lines}
        ok = len(vals) <= 1 and all(ln["calls"][c]["rc"] == 0 and ln["calls"][c]["uniform"] for ln in lines)
        v = vals.pop() if len(vals) == 1 else None
        if v is not None and v not in (full, full - victim):
            ok = False
        if dropped and v == full:
            ok = False
        dropped = dropped or v == full - victim
        consistent = consistent and ok
        per.append({"value": v, "recoveries": max((ln["calls"][c]["recoveries"] for ln in lines), default=None),
                    "ms_max_over_ranks": round(max((ln["calls"][c]["ms"] for ln in lines), default=0.0), 3)})
    out["per_call"] = per
    out["outcome"] = "aborted" if out["aborted"] else "recovered" if len(lines) == ranks - 1 else \
        "no fault hit" if len(lines) == ranks else "lost"
    out["results_consistent"] = consistent
    return out


def leg_flag(tag):
    """Flag file rank 0 writes when a rank-0 leg ends (one per torchrun job: its master
    port and agent pid)."""
    return os.path.join("/tmp", f"ftar-bench-{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}-{tag}")


def side_legs(args, rank, world, devices, rehearsal):
    """The legs rank 0 runs as other processes -- the CPU baseline (host processes), the
    configs[4] jobs (ftrun, 9 ranks) and the fabric probe (one process on every GPU) --
    BEFORE any torchrun rank touches a GPU: the other ranks wait here on a flag file
    without having imported torch.  Run after the main legs they would share the cards
    with the job's own ranks (8 + 9 GPU processes at N = 8, beyond what a box lets one
    job run on a card).  Returns (cpu, c5, xgmi) on rank 0, Nones elsewhere."""
    flag = leg_flag("side")
    if rank != 0:
        while not os.path.exists(flag):
            time.sleep(0.05)
        return None, None, None
    S = args.count * 4
    cpu = c5 = xgmi = None
    try:
        if not args.no_cpu_baseline:
            # the same schedule on this node's host cores, float32, 256 MiB per rank
            try:
                r, model = cpu_schedule("raben", world, args.count, 3)
                cpu = {"value": round(world * S / r["time_s"] / 1e9, 4), "unit": "GB/s", "cores": world,
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
            except Exception as e:
                cpu = {"value": None, "unit": "GB/s", "cores": world, "kind": "port",
                       "sample": f"failed: {str(e)[-300:]}"}
        if not args.no_c5:
            # configs[4]: N GPUs' worth of ranks + the idle spare, its own ftrun jobs
            try:
                c5 = c5_leg(world, devices, args.count, int(os.environ.get("FTAR_C5_RANKS", "9")))
            except Exception as e:
                c5 = {"error": str(e)[-500:]}
        if not args.no_xgmi:
            # the fabric (tools/xgmi_probe.hip, one process driving the job's GPUs): one
            # link one way and both ways (SURVEY.md 8d's B_link), pull vs push, copy
            # engines, the mesh's all-peers pattern; loopback in a one-GPU rehearsal
            exe = os.path.join(ROOT, "tools", "_build", "xgmi_probe")
            try:
                cp = subprocess.run([exe, str(1 if rehearsal else world)], capture_output=True, text=True,
                                    timeout=240)
                lines = [ln for ln in cp.stdout.splitlines() if ln.startswith("{")]
                xgmi = json.loads(lines[-1]) if lines else {"error": (cp.stderr or cp.stdout)[-300:],
                                                            "rc": cp.returncode}
            except Exception as e:
                xgmi = {"error": str(e)[-300:]}
    finally:
        with open(flag, "w") as f:
            f.write("done")
    return cpu, c5, xgmi


def multi(args):
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # FTAR_DEVICE pins every rank to one GPU (single-GPU rehearsal of the multi-rank path;
    # RCCL refuses two ranks on one device, so such runs use --dist-backend gloo)
    rehearsal = "FTAR_DEVICE" in os.environ  # every rank on one GPU
    # this job's GPUs (LOCAL_RANK = GPU on one node), or the one GPU of a rehearsal
    devices = [int(os.environ["FTAR_DEVICE"])] if rehearsal else list(range(world))
    cpu, c5, xgmi = side_legs(args, rank, world, devices, rehearsal)
    import torch
    import torch.distributed as dist
    ftar = load_package()
    dev = int(os.environ.get("FTAR_DEVICE", local)) % max(1, torch.cuda.device_count())
    os.environ.setdefault("FTAR_DEVICE", str(dev))  # the library opens the same device
    torch.cuda.set_device(dev)
    dist.init_process_group(backend=args.dist_backend)
    dist.barrier()
    if rank == 0:
        os.unlink(leg_flag("side"))  # every rank is past side_legs
    comm = ftar.Comm.from_env()
    comm.set_profiling(False)  # kernel events only in the profiled passes (timed_split)
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    x = torch.rand(args.count, device="cuda", generator=g) * 2 - 1
    y = torch.empty_like(x)
    S = args.count * 4
    nccl = args.dist_backend == "nccl"

    def max_over_ranks(vals):
        t = torch.tensor(vals, dtype=torch.float64)
        if nccl:
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [v.item() for v in t.cpu()]

    def timed(fn, steps=None, warmup=None):
        steps = args.steps if steps is None else steps
        warmup = args.warmup if warmup is None else warmup
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step0 = kern = syncw = drain = 0.0
        for _ in range(steps):
            fn()
            st = comm.last_stats()
            step0 += st.step0_kernel_ms
            kern += st.kernel_ms
            syncw += st.sync_wait_s
            drain += st.drain_s
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        dist.barrier()
        t, k, kall, sw, dr = max_over_ranks([t1 - t0, step0, kern, syncw, drain])
        timed.link_bytes = comm.last_stats().step0_link_bytes
        # where a call's time goes (max over ranks of each part, per call)
        timed.breakdown = {"call_ms": round(t / steps * 1e3, 4), "kernels_ms": round(kall / steps, 4),
                           "dominant_kernel_ms": round(k / steps, 4), "agree_barrier_wait_ms": round(sw / steps * 1e3, 4),
                           "stream_drain_wait_ms": round(dr / steps * 1e3, 4)}
        return t / steps, k / steps

    def timed_split(fn):
        """Per-call time with no kernel events in the timed region (the plain cost), then
        the dominant kernel's device time from a shorter profiled pass."""
        comm.set_profiling(False)
        t, _ = timed(fn)
        comm.set_profiling(True)
        _, k = timed(fn, max(3, args.steps // 4), 1)
        timed_split.breakdown = dict(timed.breakdown, profiled=True)
        return t, k

    def raben():
        rc = comm.allreduce_rabenseifner(x, y)
        assert rc == 0, rc

    def rd():
        rc = comm.recursive_doubling(x, y)
        assert rc == 0, rc

    def quick(fn, steps=3, warmup=1):
        return timed(fn, steps, warmup)[0]

    opts = (ftar.OPT_RELAY, ftar.OPT_OVERLAP, ftar.OPT_COPY_ENGINE, ftar.OPT_REDUNDANCY, ftar.OPT_MESH)
    defaults = {o: comm.get_option(o) for o in opts}

    def set_opts(vals):
        for o, v in zip(opts, vals):
            comm.set_option(o, v)

    # Exactness on this node's GPUs, every transport: integer-valued float32 inputs that
    # change from trial to trial (so a stale cached line or a read of the previous call's
    # window cannot pass), where every partial sum is an integer below 2^24 and hence
    # exact in any order.  Each rank regenerates every rank's input from its seed and sums
    # them itself: the expected result needs no collective.  Trials reuse the same buffers
    # (the peers' mappings of our send buffer are reused too).
    xe = torch.empty(args.count, device="cuda")
    ye = torch.empty_like(xe)
    want = torch.empty_like(xe)

    def int_input(out, trial, r, n):
        ge = torch.Generator(device="cuda").manual_seed(7919 * trial + r)
        out[:n].copy_(torch.randint(-1024, 1024, (n,), device="cuda", generator=ge, dtype=torch.int32))

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
    # ranks, identical on every rank) picks one.  All three give the same bits.
    selection = None
    pow2 = world & (world - 1) == 0
    if world >= 2 and not args.no_variants:
        cands = {}
        if pow2 and comm.get_option(ftar.OPT_MESH):
            cands["mesh"] = (1, 1)
        if world >= 3 and comm.get_option(ftar.OPT_RELAY):
            cands["relay2hop"] = (0, 1)
        cands["direct"] = (0, 0)
        if len(cands) > 1:
            times, inexact = {}, []
            for name, (m, r) in cands.items():
                comm.set_option(ftar.OPT_MESH, m)
                comm.set_option(ftar.OPT_RELAY, r)
                # a transport that is not bit-exact on this node never times the headline
                if max_over_ranks([exact_ok(comm.allreduce_rabenseifner, trials=(0,))])[0]:
                    inexact.append(name)
                    continue
                times[name] = quick(raben)
            if times:
                chosen = min(times, key=times.get)
                comm.set_option(ftar.OPT_MESH, cands[chosen][0])
                comm.set_option(ftar.OPT_RELAY, cands[chosen][1])
            else:  # every one failed: keep the defaults, exact_on_node reports it
                chosen = None
                comm.set_option(ftar.OPT_MESH, defaults[ftar.OPT_MESH])
                comm.set_option(ftar.OPT_RELAY, defaults[ftar.OPT_RELAY])
            selection = {f"{k}_ms": round(t * 1e3, 4) for k, t in times.items()}
            selection["chosen"] = chosen
            selection["inexact"] = inexact

    t_rb, k_rb = timed_split(raben)
    step0_bytes = timed.link_bytes
    breakdown = timed_split.breakdown
    relayed = comm.last_stats().relayed_steps > 0
    meshed = comm.last_stats().mesh_steps > 0
    oneshot = comm.last_stats().mesh_steps == 1  # the mesh's one-launch form (p = 2, small vectors)
    transport = "mesh-oneshot" if oneshot else "mesh" if meshed else "relay2hop" if relayed else "direct"
    chosen_opts = {o: comm.get_option(o) for o in opts}
    # correctness spot check against torch.distributed's all_reduce on the same inputs
    # (fp32, different reduction order: |err| <= log2(p) * 2^-24 * sum|x_i|)
    ref = x.clone() if nccl else x.cpu()
    dist.all_reduce(ref)
    raben()
    err = (y.cpu() - ref.cpu()).abs().max().item()
    # the reference drivers' case (buffer[i] = rank, int32 SUM): closed-form checksum
    # sum_i result[i] % 17 = ((p (p-1) / 2) % 17) * count  (analysis/check_fault.py:62-67)
    xi = torch.full((args.count,), rank, dtype=torch.int32, device="cuda")
    yi = torch.empty_like(xi)
    assert comm.allreduce_rabenseifner(xi, yi) == 0
    cks_raben = int((yi.to(torch.int64) % 17).sum().item())
    assert comm.recursive_doubling(xi, yi) == 0
    cks_rd = int((yi.to(torch.int64) % 17).sum().item())
    cks_want = ((world * (world - 1) // 2) % 17) * args.count
    del xi, yi
    # The reference's own data movement, first class: pairwise pulls, step by step, one
    # link per step, with the step-0 full-vector exchange kept (its tmp redundancy,
    # raben/rabenseifner.c:206-211) even where no handler can use it.
    set_opts((0, 0, 0, 1, 0))
    t_ref, k_ref = timed_split(raben)
    set_opts([chosen_opts[o] for o in opts])
    # recursive doubling has no mesh form (it can recover at any p): relay or direct
    rd_selection = None
    relay_for_raben = comm.get_option(ftar.OPT_RELAY)
    if world >= 3 and not args.no_variants:
        comm.set_option(ftar.OPT_RELAY, 1)
        t_r = quick(rd)
        comm.set_option(ftar.OPT_RELAY, 0)
        t_d = quick(rd)
        comm.set_option(ftar.OPT_RELAY, 1 if t_r <= t_d else 0)
        rd_selection = {"relay2hop_ms": round(t_r * 1e3, 4), "direct_ms": round(t_d * 1e3, 4),
                        "chosen": "relay2hop" if t_r <= t_d else "direct"}
    t_rd, k_rd = timed_split(rd)
    comm.set_option(ftar.OPT_RELAY, relay_for_raben)
    # the same schedules over the other transports
    transports = {}
    if not args.no_variants:
        # mesh: one-hop reduce-scatter + allgather (power-of-two p, no spare); relay2hop:
        # the step-by-step schedule striped over 2-hop paths; direct: one pull kernel per
        # step; direct_serial: plus the step-0 copy inline; copy_engine: hipMemcpyAsync of
        # the partner's window + a local reduce kernel; relay_full_exchange: the relay with
        # the reference's step-0 full exchange
        variants = (("mesh", (1, 1, 0, 0, 1)), ("relay2hop", (1, 1, 0, 0, 0)), ("direct", (0, 1, 0, 0, 0)),
                    ("direct_serial", (0, 0, 0, 0, 0)), ("copy_engine", (0, 1, 1, 0, 0)),
                    ("relay_full_exchange", (1, 1, 0, 1, 0)))
        for name, vals in variants:
            if name == "mesh" and not pow2:
                continue
            set_opts(vals)
            tv, kv = timed_split(raben)
            lb = timed.link_bytes
            tv_rd, _ = timed(rd) if name in ("relay2hop", "direct", "copy_engine") else (None, None)
            transports[name] = {"raben_ms": round(tv * 1e3, 4), "raben_algbw_GBps": round(S / tv / 1e9, 2),
                                "step0_kernel_ms": round(kv, 4), "step0_link_bytes": lb,
                                "step0_pull_GBps": round(lb / (kv * 1e-3) / 1e9, 2) if kv > 0 else None}
            if tv_rd:
                transports[name].update({"rd_ms": round(tv_rd * 1e3, 4), "rd_algbw_GBps": round(S / tv_rd / 1e9, 2)})
        set_opts([chosen_opts[o] for o in opts])
    # Exactness of every transport on this node (helpers above the selection)
    checks = [("chosen", [chosen_opts[o] for o in opts], comm.allreduce_rabenseifner, None),
              ("reference_shape", (0, 0, 0, 1, 0), comm.allreduce_rabenseifner, None),
              ("rd", [chosen_opts[o] for o in opts], comm.recursive_doubling, None),
              ("chosen_64KiB", [chosen_opts[o] for o in opts], comm.allreduce_rabenseifner, 16384)]
    if not args.no_variants:
        checks += [(name, vals, comm.allreduce_rabenseifner, None) for name, vals in
                   (("mesh", (1, 1, 0, 0, 1)), ("relay2hop", (1, 1, 0, 0, 0)), ("direct", (0, 1, 0, 0, 0)),
                    ("copy_engine", (0, 1, 1, 0, 0))) if pow2 or name != "mesh"]
        checks += [("rd_relay", (1, 1, 0, 0, 0), comm.recursive_doubling, None),
                   ("rd_direct", (0, 1, 0, 0, 0), comm.recursive_doubling, None)]
    comm.set_profiling(False)
    fails = []
    for name, vals, fn, n in checks:
        set_opts(vals)
        if name == "rd" and rd_selection:  # the transport the RD timing chose
            comm.set_option(ftar.OPT_RELAY, int(rd_selection["chosen"] == "relay2hop"))
        fails.append(exact_ok(fn, n=n))
    set_opts([chosen_opts[o] for o in opts])
    comm.set_profiling(True)
    fails = max_over_ranks(fails)
    exact = {"inputs": "integer-valued float32 in [-1024, 1024), new per trial, 2 trials per transport; expected "
                       "sum regenerated on every rank (exact in any order)",
             "all_exact": all(f == 0 for f in fails)}
    exact.update({name: f == 0 for (name, _, _, _), f in zip(checks, fails)})
    del xe, ye, want
    # Per-call time over message sizes (max over ranks), 4 B .. 256 MiB, with the chosen
    # transport, next to RCCL's all_reduce on the same sizes: the FT/vendor curve of the
    # reference's compare campaign (slurm/test_compare.slurm:27-50, check_compare.py),
    # plus the fixed cost per call and the one-shot threshold (FTAR_ONESHOT_MAX)
    sizes = {}
    if not args.no_variants:
        comm.set_profiling(False)  # no kernel events: the plain per-call cost
        oneshot_max = comm.get_option(ftar.OPT_ONESHOT_MAX)
        z = x.clone() if nccl else None
        n = 1
        while n <= args.count:
            steps, warm = (20, 3) if n <= (1 << 22) else (5, 2)
            row = {"bytes": 4 * n}
            for name, fn, extra in (("raben", comm.allreduce_rabenseifner, None),
                                    ("raben_no_oneshot", comm.allreduce_rabenseifner, 0),
                                    ("rd", comm.recursive_doubling, None)):
                if extra is not None:
                    if not (pow2 and comm.get_option(ftar.OPT_MESH) and oneshot_max > 0) or \
                            (world > 2 and 4 * n > oneshot_max):
                        continue
                    comm.set_option(ftar.OPT_ONESHOT_MAX, extra)

                def call(fn=fn, n=n):
                    rc = fn(x, y, count=n)
                    assert rc == 0, rc

                row[name + "_us"] = round(quick(call, steps=steps, warmup=warm) * 1e6, 2)
                comm.set_option(ftar.OPT_ONESHOT_MAX, oneshot_max)
            if z is not None:
                zn = z[:n]
                row["rccl_us"] = round(quick(lambda: dist.all_reduce(zn), steps=steps, warmup=warm) * 1e6, 2)
                row["raben_over_rccl"] = round(row["raben_us"] / row["rccl_us"], 3)
            sizes[str(4 * n)] = row
            n *= 2
        comm.set_profiling(True)
    # end-to-end with host buffers: pinned H2D + device Allreduce + D2H (never the value)
    xh = x.cpu().pin_memory()
    yh = torch.empty_like(xh).pin_memory()

    def raben_host():
        rc = comm.allreduce_rabenseifner_host(xh, yh)
        assert rc == 0, rc

    t_e2e, _ = timed(raben_host, 3, 1)
    t_nc = None
    if nccl:
        zz = x.clone()
        t_nc, _ = timed(lambda: dist.all_reduce(zz))

    L = world.bit_length() - 1
    r = 1 << L  # ranks in the power-of-two core: the receivers of every exchange step
    # Link bytes per rank per direction.  The reference's FT Raben moves
    # (2.5 - 2^(1-L)) S: its step 0 exchanges the full vector, half of it only as
    # recovery data.  At power-of-two p no handler can use that half (they all abort
    # without a spare), so the build skips it there and moves classic Rabenseifner's
    # 2 (1 - 2^-L) S.  A relayed step moves 2/r of its window per link (two phases
    # over r-1 links); a direct step moves it over one link.
    ft_bytes = (2.5 - 2.0 ** (1 - L)) * S
    classic = 2 * (1 - 2.0 ** -L) * S
    keep = world != r or comm.get_option(ftar.OPT_REDUNDANCY) != 0
    sched_bytes = ft_bytes if keep else classic
    if oneshot:
        # every peer's whole vector over its own link: S per link (= 2 S / p at p = 2)
        t_roof = S / (XGMI_LINK_GBS * 1e9)
    elif meshed:
        # one hop over p - 1 links: S/p per link for each of reduce-scatter and allgather
        t_roof = 2.0 * S / world / (XGMI_LINK_GBS * 1e9)
    elif relayed:
        t_roof = 2.0 / r * sched_bytes / (XGMI_LINK_GBS * 1e9)
    elif comm.get_option(ftar.OPT_OVERLAP) != 0:
        t_roof = classic / (XGMI_LINK_GBS * 1e9)
    else:
        t_roof = sched_bytes / (XGMI_LINK_GBS * 1e9)
    t_survey = ft_bytes / (XGMI_LINK_GBS * 1e9)  # the FT schedule on one link per step
    links = (world - 1) if meshed else (r - 1) if relayed else 1
    peak = links * XGMI_LINK_GBS
    achieved = step0_bytes / (k_rb * 1e-3) / 1e9 if k_rb > 0 else None  # RS step-0 kernels' pulled bytes

    def frac(x):
        # a one-GPU rehearsal has no xGMI link in the path (every "peer" read is local
        # HBM shared by all ranks): link-roofline fractions would mix yardsticks
        return None if rehearsal else round(x, 4)
    # Link calibration ("B_link = the calibrated single-link unidirectional
    # GB/s with both directions loaded"): the direct transport's RS step 0 is one kernel
    # per rank pulling the partner's half over ONE link while the partner pulls ours, so
    # its pulled bytes / its duration is that figure, measured in this job.
    link_cal = None
    dcal = transports.get("direct", {})
    probe = (xgmi or {}).get("patterns", {}).get("pull1_bidir", {})
    if dcal.get("step0_pull_GBps") or probe.get("GBps_per_link"):
        # the probe's plain copy over one link, both ways, where it ran on the node;
        # otherwise the direct transport's step-0 pull
        b = probe.get("GBps_per_link") if probe.get("ok") and probe.get("GBps_per_link") else dcal.get("step0_pull_GBps")
        link_cal = {"single_link_GBps": b, "spec_GBps": XGMI_LINK_GBS, "frac_of_spec": frac(b / XGMI_LINK_GBS),
                    "source": "xgmi_probe pull1_bidir" if b == probe.get("GBps_per_link") else "direct step 0",
                    "direct_step0": {"kernel": "direct transport, Raben RS step 0: pull the partner's half + reduce, "
                                               "both directions loaded", "bytes": dcal.get("step0_link_bytes"),
                                     "kernel_ms": dcal.get("step0_kernel_ms"),
                                     "pull_GBps": dcal.get("step0_pull_GBps")}}
    schedule = {
        "mesh-oneshot": "Rabenseifner, one-shot mesh: every block in its owner's reduction tree in one launch "
                        "(power-of-two p, no spare)",
        "mesh": "Rabenseifner, one-hop mesh: reduce-scatter as one tree kernel over p-1 peer pulls, allgather as "
                "one multi-source pull (power-of-two p, no spare; same reduction tree as recursive halving)",
        "relay2hop": "Rabenseifner, step by step (recursive halving + doubling), each exchange striped over 2-hop "
                     "relays",
        "direct": "Rabenseifner, step by step (recursive halving + doubling), one pairwise pull per step",
    }[transport]
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(world * S / t_rb / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_rb * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uniform[-1,1), HBM-resident",
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
            "reference_shape": {
                "schedule": "Rabenseifner step by step, pairwise pulls (one xGMI link per step), step-0 full-vector "
                            "exchange kept (raben/rabenseifner.c:206-211)",
                "value": round(world * S / t_ref / 1e9, 2), "ms_per_step": round(t_ref * 1e3, 4),
                "algbw_GBps": round(S / t_ref / 1e9, 2), "step0_kernel_ms": round(k_ref, 4),
                "survey_ft_roofline_ms": round(t_survey * 1e3, 3),
                "frac_of_survey_roofline": frac(t_survey / t_ref)},
            "schedule_link_roofline": {"schedule_bytes_per_rank": sched_bytes, "link_GBps": XGMI_LINK_GBS,
                                       "links_per_step": links, "t_roof_ms": round(t_roof * 1e3, 3),
                                       "frac": frac(t_roof / t_rb),
                                       # the same roofline priced at the calibrated link rate
                                       "frac_calibrated_link": frac(t_roof * XGMI_LINK_GBS
                                                                    / link_cal["single_link_GBps"] / t_rb)
                                       if link_cal else None},
            "link_calibration": link_cal,
            "xgmi_probe": xgmi,
            "roofline": {"bound": "xgmi", "achieved": round(achieved, 1) if achieved else None,
                         "peak": peak, "unit": "GB/s",
                         "frac": frac(achieved / peak) if achieved else None,
                         "rehearsal": rehearsal,
                         # HBM bytes per launch from PMC exist for the one-GPU rehearsal only
                         # (every peer on this device); on the node the peer reads hit the
                         # peers' HBM and the counters of one device miss them
                         "traffic": pmc_traffic(f"mesh_tree_p{world}_rehearsal") if rehearsal and meshed
                         and not oneshot else None,
                         "traffic_note": "PMC counters of a peer-reading kernel are per device; not collected on "
                                         "the 8-GPU node (profiles/pmc_summary.json has the one-GPU rehearsal's: "
                                         "tree and allgather kernels within 0.02 % of their algorithmic bytes)",
                         "kernel": ("Raben one-shot mesh: tree_batch_kernel, every block in its owner's tree"
                                    if oneshot
                                    else "Raben mesh reduce-scatter: tree_kernel over p-1 one-hop pulls" if meshed
                                    else "Raben RS step 0, both relay phases (stripes pulled over r-1 links)" if relayed
                                    else "Raben RS step 0 reduce half (pull partner's half, reduce into W)"),
                         "algorithmic_bytes_per_launch": step0_bytes, "kernel_ms": round(k_rb, 4)},
            "e2e_host_buffers": {"ms_per_step": round(t_e2e * 1e3, 3), "algbw_GBps": round(S / t_e2e / 1e9, 2)},
            "rd": {"ms_per_step": round(t_rd * 1e3, 4), "algbw_GBps": round(S / t_rd / 1e9, 2),
                   "value": round(world * S / t_rd / 1e9, 2),
                   "step0_kernel_ms": round(k_rd, 4), "transport_selection": rd_selection},
            "rccl_allreduce": ({"ms_per_step": round(t_nc * 1e3, 4), "algbw_GBps": round(S / t_nc / 1e9, 2),
                                "value": round(world * S / t_nc / 1e9, 2)} if t_nc else None),
            "transport_selection": selection,
            "transports": transports,
            "size_sweep_us": sizes,
            "max_abs_err_vs_rccl": err,
            "int32_rank_checksum_ok": {"raben": cks_raben == cks_want, "rd": cks_rd == cks_want},
            "exact_on_node": exact,
            "c5_single_kill": c5,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
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
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
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
