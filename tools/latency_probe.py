"""Where the fixed cost of a small Allreduce goes, ranks sharing one GPU (ftrun job):
median per-call wall time, the part spent draining the stream, and the device time of
the exchange kernel (hipEvents), next to a plain torch launch + synchronize issued by
every rank at once (the device round trip without the library).

    fault-tolerant_amd/bin/ftrun -np 2 --devmap 0,0 python tools/latency_probe.py [out.json]

LAT_COUNT=<elements> (default 1024 float32 = 4 KiB) times mid-size calls, e.g. 524288 (2 MiB)
or 2097152 (8 MiB): there RD queues steps 1.. and the mesh its allgather behind gates
relayed through device memory (FTAR_GATE_MAX), rows *_nogate launch after the barriers.
"""
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def med(v):
    v = sorted(v)
    return round(v[len(v) // 2] * 1e6, 1)


def main():
    rank = int(os.environ["FTAR_RANK"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    count = int(os.environ.get("LAT_COUNT", "1024"))
    iters = int(os.environ.get("LAT_ITERS", "200" if count <= 65536 else "60"))
    x = torch.rand(count, device="cuda")
    y = torch.empty_like(x)
    res = {"ranks": int(os.environ["FTAR_SIZE"]), "bytes": 4 * count}
    # plain device round trip, every rank at once
    ts = []
    for _ in range(200):
        comm.barrier()
        t0 = time.perf_counter()
        y.copy_(x)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res["torch_launch_sync_us"] = med(ts)
    ts = []
    for _ in range(200):
        comm.barrier()
        t0 = time.perf_counter()
        comm.barrier()
        ts.append(time.perf_counter() - t0)
    res["ftar_barrier_us"] = med(ts)
    for prof in (0, 1):
        comm.set_profiling(bool(prof))
        # raben_oneshot: its launch queued ahead of the barrier behind a gate (FTAR_OPT_GATE,
        # the default); raben_oneshot_nogate: launched after the barrier (round 3's first form)
        for name, fn, limit, gate in (("raben_oneshot", comm.allreduce_rabenseifner, 1 << 20, 1),
                                      ("raben_oneshot_nogate", comm.allreduce_rabenseifner, 1 << 20, 0),
                                      ("raben_mesh", comm.allreduce_rabenseifner, 0, 1),
                                      ("raben_mesh_nogate", comm.allreduce_rabenseifner, 0, 0),
                                      ("rd", comm.recursive_doubling, 0, 1),
                                      ("rd_nogate", comm.recursive_doubling, 0, 0)):
            comm.set_option(ftar.OPT_ONESHOT_MAX, limit)
            comm.set_option(ftar.OPT_GATE, gate)
            # mid-size gates are off by default (FTAR_OPT_GATE_MAX = 1 MiB): on for the gated rows
            comm.set_option(ftar.OPT_GATE_MAX, 16 << 20 if gate else 1 << 20)
            for _ in range(5):
                assert fn(x, y) == 0
            wall, drain, sync, kern, cwall, gated, holds = [], [], [], [], [], [], []
            for _ in range(iters):
                comm.barrier()
                t0 = time.perf_counter()
                assert fn(x, y) == 0
                wall.append(time.perf_counter() - t0)
                st = comm.last_stats()
                drain.append(st.drain_s)
                sync.append(st.sync_wait_s)
                kern.append(st.step0_kernel_ms * 1e-3)
                cwall.append(st.wall_s)
                gated.append(st.gated_launches - st.gated_skips)
                holds.append(st.gate_holds)
            key = name + ("_profiled" if prof else "")
            # wall: the Python call; c_wall: inside the C entry point (ftar_stats wall_s,
            # what a C caller of include/ftar.h pays, minus the argument checks)
            res[key] = {"wall_us": med(wall), "c_wall_us": med(cwall), "drain_us": med(drain),
                        "sync_wait_us": med(sync), "gated_calls": sum(1 for g in gated if g),
                        # gated launches given up at a barrier that waited past FTAR_GATE_HOLD_US: a
                        # row where most are given up measures the hold, not the gate
                        "gate_holds": sum(holds)}
            if prof:
                res[key]["step0_kernel_us"] = med(kern)
    comm.set_option(ftar.OPT_ONESHOT_MAX, 1 << 20)
    comm.set_option(ftar.OPT_GATE, 1)
    if rank == 0:
        print(json.dumps(res), flush=True)
        if len(sys.argv) > 1:
            with open(sys.argv[1], "w") as f:
                json.dump(res, f)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
