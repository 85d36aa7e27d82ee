"""Per-call time of both FT schedules over message sizes (the shape of the reference's
compare campaign, slurm/test_compare.slurm:27-50: 4 B .. 2^27 ints), device-resident.

Run as the ranks of one ftrun job (every rank on the GPU ftrun assigns it):

    fault-tolerant_amd/bin/ftrun -np 4 --devmap 0,0,0,0 python tools/size_sweep.py [out.json]

Each size: 3 warm-up calls, then `reps` timed calls, each started right after an
ftar_barrier; rank 0 reports the median of its per-call wall times (the ranks leave the
barrier together, so this is one Allreduce from a common start).  Float32 SUM,
uniform inputs.  Up to 4 MiB (every size at 2 ranks) the two-launch mesh is timed too ("raben2", one-shot off),
beside the default (one-shot up to FTAR_ONESHOT_MAX).
"""
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    rank = int(os.environ["FTAR_RANK"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    sizes = [1 << k for k in range(0, 27, 2)] + [1 << 26]
    res = []
    for n in sizes:
        x = torch.rand(n, device="cuda") * 2 - 1
        y = torch.empty_like(x)
        reps = 50 if n <= (1 << 20) else 10
        row = {"count": n, "bytes": 4 * n}
        oneshot = comm.get_option(ftar.OPT_ONESHOT_MAX)
        variants = [("raben", comm.allreduce_rabenseifner, oneshot), ("rd", comm.recursive_doubling, oneshot)]
        if 4 * n <= (4 << 20) or int(os.environ["FTAR_SIZE"]) == 2:
            variants.append(("raben2", comm.allreduce_rabenseifner, 0))
        for name, fn, limit in variants:
            comm.set_option(ftar.OPT_ONESHOT_MAX, limit)
            for _ in range(3):
                assert fn(x, y) == 0
            ts = []
            for _ in range(reps):
                comm.barrier()
                t0 = time.perf_counter()
                assert fn(x, y) == 0
                ts.append(time.perf_counter() - t0)
            ts.sort()
            st = comm.last_stats()
            row[name + "_us"] = round(ts[len(ts) // 2] * 1e6, 1)
            row[name + "_syncs"] = st.syncs
            row[name + "_sync_wait_us"] = round(st.sync_wait_s * 1e6, 1)
            row[name + "_drain_us"] = round(st.drain_s * 1e6, 1)
            row[name + "_launches"] = st.mesh_steps
        comm.set_option(ftar.OPT_ONESHOT_MAX, oneshot)
        res.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)
    if rank == 0 and out:
        with open(out, "w") as f:
            json.dump({"ranks": int(os.environ["FTAR_SIZE"]), "rows": res}, f)
    comm.finalize()


if __name__ == "__main__":
    main()
