#!/usr/bin/env python3
"""bench.py -- Allreduce GB/s (device-resident, float32 SUM) of the MI355X-native
fault-tolerant Allreduce.

  python bench.py [--gpus 1] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

N = 1: the single-GPU workload of BASELINE.json configs[1] -- the local-reduce HIP
       kernel (MPI_Reduce_local, the per-step bucket reduction) on two 256 MiB float32
       vectors.  One step = one kernel launch.  HBM-bound.
N > 1: configs[3] -- fault-tolerant Rabenseifner Allreduce of a 256 MiB float32 vector
       per rank, one rank per GPU, exchanges pulled over xGMI (weak scaling: every rank
       contributes one 256 MiB vector).  One step = one Allreduce.  Recursive doubling
       (configs[2]) and RCCL's all_reduce on the same buffers are reported beside it.

value = (input vectors summed x bytes per vector) / time per step, whole job:
        N=1: 2 x 256 MiB per launch; N>1: N x 256 MiB per Allreduce.
Data are synthetic (uniform [-1, 1)), inputs resident in HBM before timing starts.
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
COUNT = 1 << 26              # 256 MiB of float32 per vector
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 76.8         # one xGMI link, one direction (153.6 GB/s bidirectional spec)
METRIC = "Allreduce GB/s (device-resident, float32 SUM) at 1/2/4/8 MI355X"


def load_package():
    path = os.path.join(ROOT, "fault-tolerant_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("ftar_amd", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ftar_amd"] = mod
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


def single(args):
    import torch
    ftar = load_package()
    ftar.lib()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(42)
    x = torch.rand(args.count, device="cuda", generator=g) * 2 - 1
    y = torch.rand(args.count, device="cuda", generator=g) * 2 - 1
    ftar.set_reduce_variant(args.variant)
    for _ in range(args.warmup):
        ftar.reduce_local(x, y)
    torch.cuda.synchronize()
    if args.timing == "launch":
        # an event pair around every launch: per-launch kernel time, at the cost of two
        # timestamp markers between consecutive kernels in the timed region
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record()
            ftar.reduce_local(x, y)  # launched on torch's current stream, the one the events see
            e1.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        k_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / args.steps
    else:
        # one event pair around the whole timed region: the average launch duration
        # includes the kernel-to-kernel boundaries, nothing is inserted between launches
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(args.steps):
            ftar.reduce_local(x, y)
        e1.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        k_ms = e0.elapsed_time(e1) / args.steps
    ms_step = (t1 - t0) * 1e3 / args.steps
    S = args.count * 4
    achieved = 3 * S / (k_ms * 1e-3) / 1e9
    out = {
        "metric": METRIC, "value": round(2 * S / (ms_step * 1e-3) / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic uniform[-1,1), HBM-resident",
        "config": {"workload": "configs[1]: local-reduce HIP kernel (MPI_Reduce_local), 2 x 256 MiB float32 SUM, "
                               "1 MI355X", "count": args.count, "kernel_variant": args.variant,
                   "timing": args.timing},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic("reduce_local_c2_lds" if args.variant == 1 else "reduce_local_c2"),
                     "kernel": "reduce_lds_kernel<float,SUM>" if args.variant == 1 else "segment_kernel<float,SUM>",
                     "algorithmic_bytes_per_launch": 3 * S,
                     "kernel_ms": round(k_ms, 4)},
    }
    out["e2e"] = e2e_local(ftar, args.count)
    out["cpu_baseline"] = None if args.no_cpu_baseline else cpu_baseline_local_reduce()
    print(json.dumps(out), flush=True)


def e2e_local(ftar, count, iters=5):
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
    return {"h2d_GBps": round(2 * S * iters / ts["h2d"] / 1e9, 2), "d2h_GBps": round(S * iters / ts["d2h"] / 1e9, 2),
            "ms": round(ts["total"] * 1e3 / iters, 3),
            "GBps": round(2 * S * iters / ts["total"] / 1e9, 2)}


def multi(args):
    import torch
    import torch.distributed as dist
    ftar = load_package()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # FTAR_DEVICE pins every rank to one GPU (single-GPU rehearsal of the multi-rank path;
    # RCCL refuses two ranks on one device, so such runs use --dist-backend gloo)
    dev = int(os.environ.get("FTAR_DEVICE", local)) % max(1, torch.cuda.device_count())
    os.environ.setdefault("FTAR_DEVICE", str(dev))  # the library opens the same device
    torch.cuda.set_device(dev)
    dist.init_process_group(backend=args.dist_backend)
    comm = ftar.Comm.from_env()
    comm.set_profiling(True)
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    x = torch.rand(args.count, device="cuda", generator=g) * 2 - 1
    y = torch.empty_like(x)
    S = args.count * 4

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step0 = 0.0
        for _ in range(args.steps):
            fn()
            step0 += comm.last_stats().step0_kernel_ms
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        dist.barrier()
        t = torch.tensor([t1 - t0, step0], dtype=torch.float64)
        if args.dist_backend == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        timed.link_bytes = comm.last_stats().step0_link_bytes
        return t[0].item() / args.steps, t[1].item() / args.steps

    def raben():
        rc = comm.allreduce_rabenseifner(x, y)
        assert rc == 0, rc

    def rd():
        rc = comm.recursive_doubling(x, y)
        assert rc == 0, rc

    def quick(fn, steps=3, warmup=1):
        saved = (args.steps, args.warmup)
        args.steps, args.warmup = steps, warmup
        try:
            return timed(fn)[0]
        finally:
            args.steps, args.warmup = saved

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
            times = {}
            for name, (m, r) in cands.items():
                comm.set_option(ftar.OPT_MESH, m)
                comm.set_option(ftar.OPT_RELAY, r)
                times[name] = quick(raben)
            chosen = min(times, key=times.get)
            comm.set_option(ftar.OPT_MESH, cands[chosen][0])
            comm.set_option(ftar.OPT_RELAY, cands[chosen][1])
            selection = {f"{k}_ms": round(t * 1e3, 4) for k, t in times.items()}
            selection["chosen"] = chosen

    t_rb, k_rb = timed(raben)
    step0_bytes = timed.link_bytes
    relayed = comm.last_stats().relayed_steps > 0
    meshed = comm.last_stats().mesh_steps > 0
    oneshot = comm.last_stats().mesh_steps == 1  # the mesh's one-launch form (p = 2, small vectors)
    # correctness spot check against torch.distributed's all_reduce on the same inputs
    # (fp32, different reduction order: |err| <= log2(p) * 2^-24 * sum|x_i|)
    ref = x.clone() if args.dist_backend == "nccl" else x.cpu()
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
    t_rd, k_rd = timed(rd)
    comm.set_option(ftar.OPT_RELAY, relay_for_raben)
    # the same schedules over plain pairwise exchanges (one link per step), with and
    # without the background-stream redundancy copy -- the reference's transport shape
    transports = {}
    if not args.no_variants:
        opts = (ftar.OPT_RELAY, ftar.OPT_OVERLAP, ftar.OPT_COPY_ENGINE, ftar.OPT_REDUNDANCY, ftar.OPT_MESH)
        defaults = {o: comm.get_option(o) for o in opts}
        # mesh: one-hop reduce-scatter + allgather (power-of-two p, no spare); relay2hop:
        # the step-by-step schedule striped over 2-hop paths; direct: one pull kernel per
        # step; direct_serial: plus the step-0 copy inline; copy_engine: hipMemcpyAsync of
        # the partner's window + a local reduce kernel; reference_shape: pairwise, inline,
        # with the step-0 full exchange even where no handler can use it (the reference's
        # data movement); relay_full_exchange: the relay with that full exchange
        variants = (("mesh", (1, 1, 0, 0, 1)), ("relay2hop", (1, 1, 0, 0, 0)), ("direct", (0, 1, 0, 0, 0)),
                    ("direct_serial", (0, 0, 0, 0, 0)), ("copy_engine", (0, 1, 1, 0, 0)),
                    ("reference_shape", (0, 0, 0, 1, 0)), ("relay_full_exchange", (1, 1, 0, 1, 0)))
        for name, vals in variants:
            for o, v in zip(opts, vals):
                comm.set_option(o, v)
            tv, _ = timed(raben)
            tv_rd, _ = timed(rd) if name in ("relay2hop", "direct", "copy_engine") else (None, None)
            transports[name] = {"raben_ms": round(tv * 1e3, 4), "raben_algbw_GBps": round(S / tv / 1e9, 2)}
            if tv_rd:
                transports[name].update({"rd_ms": round(tv_rd * 1e3, 4), "rd_algbw_GBps": round(S / tv_rd / 1e9, 2)})
        for o, v in defaults.items():
            comm.set_option(o, v)
    # per-call time over message sizes on the node (max over ranks), with the chosen
    # transport: the fixed cost per call and the one-shot threshold (FTAR_ONESHOT_MAX)
    # measured one rank per GPU instead of estimated from the one-GPU rehearsals
    sizes = {}
    if not args.no_variants:
        comm.set_profiling(False)  # no kernel events: the plain per-call cost
        oneshot_max = comm.get_option(ftar.OPT_ONESHOT_MAX)
        for n in (1 << 8, 1 << 14, 1 << 18, 1 << 20, 1 << 22):
            if n > args.count:
                continue
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

                row[name + "_us"] = round(quick(call, steps=20, warmup=3) * 1e6, 2)
                comm.set_option(ftar.OPT_ONESHOT_MAX, oneshot_max)
            sizes[str(4 * n)] = row
        comm.set_profiling(True)
    # end-to-end with host buffers: pinned H2D + device Allreduce + D2H (never the value)
    xh = x.cpu().pin_memory()
    yh = torch.empty_like(xh).pin_memory()

    def raben_host():
        rc = comm.allreduce_rabenseifner_host(xh, yh)
        assert rc == 0, rc

    saved = (args.steps, args.warmup)
    args.steps, args.warmup = 3, 1
    t_e2e, _ = timed(raben_host)
    args.steps, args.warmup = saved
    t_nc = None
    if args.dist_backend == "nccl":
        z = x.clone()

        def rccl():
            dist.all_reduce(z)

        t_nc, _ = timed(rccl)
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
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(world * S / t_rb / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_rb * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uniform[-1,1), HBM-resident",
            "config": {"workload": "configs[3]: fault-tolerant Rabenseifner Allreduce, 256 MiB float32 SUM per "
                                   "rank, one rank per MI355X, pull exchanges over xGMI",
                       "count": args.count, "parallelism": f"{world} ranks"},
            "algbw_GBps": round(S / t_rb / 1e9, 2),
            "transport": "mesh-oneshot" if oneshot else "mesh" if meshed else "relay2hop" if relayed else "direct",
            "schedule_link_roofline": {"schedule_bytes_per_rank": sched_bytes, "link_GBps": XGMI_LINK_GBS,
                                       "links_per_step": links, "t_roof_ms": round(t_roof * 1e3, 3),
                                       "frac": round(t_roof / t_rb, 4),
                                       "survey_ft_roofline_ms": round(t_survey * 1e3, 3),
                                       "frac_of_survey_roofline": round(t_survey / t_rb, 4)},
            "roofline": {"bound": "xgmi", "achieved": round(achieved, 1) if achieved else None,
                         "peak": peak, "unit": "GB/s",
                         "frac": round(achieved / peak, 4) if achieved else None, "traffic": None,
                         "kernel": ("Raben one-shot mesh: tree_batch_kernel, every block in its owner's tree"
                                    if oneshot
                                    else "Raben mesh reduce-scatter: tree_kernel over p-1 one-hop pulls" if meshed
                                    else "Raben RS step 0, both relay phases (stripes pulled over r-1 links)" if relayed
                                    else "Raben RS step 0 reduce half (pull partner's half, reduce into W)"),
                         "algorithmic_bytes_per_launch": step0_bytes, "kernel_ms": round(k_rb, 4)},
            "e2e_host_buffers": {"ms_per_step": round(t_e2e * 1e3, 3), "algbw_GBps": round(S / t_e2e / 1e9, 2)},
            "rd": {"ms_per_step": round(t_rd * 1e3, 4), "algbw_GBps": round(S / t_rd / 1e9, 2),
                   "step0_kernel_ms": round(k_rd, 4), "transport_selection": rd_selection},
            "rccl_allreduce": ({"ms_per_step": round(t_nc * 1e3, 4), "algbw_GBps": round(S / t_nc / 1e9, 2)}
                               if t_nc else None),
            "transport_selection": selection,
            "transports": transports,
            "size_sweep_us": sizes,
            "max_abs_err_vs_rccl": err,
            "int32_rank_checksum_ok": {"raben": cks_raben == cks_want, "rd": cks_rd == cks_want},
            "cpu_baseline": None,
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
    ap.add_argument("--variant", type=int, default=1, help="local-reduce kernel: 0 register, 1 LDS-DMA (default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing", choices=["region", "launch"], default="region",
                    help="N=1 kernel time: events around the timed region, or around every launch")
    ap.add_argument("--no-variants", action="store_true", help="N>1: skip the direct-transport comparison")
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
