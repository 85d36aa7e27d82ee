"""Per-call time when the caller cycles its send buffer through K distinct allocations (a
bucketed all-reduce: one buffer per bucket), against the peers' mapping cache of the exported
inputs (FTAR_UCACHE allocations per peer, ftar_comm.c `peer_sbuf`): a buffer outside the cache
costs one import per peer, and evicting one costs a close (tools/ipc_probe.hip's capacity
phase: ~0.4 ms per hipIpcCloseMemHandle).

    fault-tolerant_amd/bin/ftrun -np 4 --devmap 0,0,0,0 python tools/ucache_probe.py [out.json]

Float32 SUM, 4 Mi elements (16 MiB, one allocation each) per buffer; for each K: one warm-up
pass over the K buffers, then `passes` timed passes, every call started after an ftar_barrier;
rank 0 reports the median per-call wall time and the exactness of the last result.
"""
import importlib.util
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    rank = int(os.environ["FTAR_RANK"])
    size = int(os.environ["FTAR_SIZE"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    n = 1 << 22
    res = []
    for k in (1, 4, 5, 8, 16):
        xs = [torch.full((n,), float(rank + 1 + 100 * i), device="cuda") for i in range(k)]
        y = torch.empty(n, device="cuda")
        for x in xs:
            assert comm.allreduce_rabenseifner(x, y) == 0
        ts = []
        passes = 6
        for _ in range(passes):
            for x in xs:
                comm.barrier()
                t0 = time.perf_counter()
                assert comm.allreduce_rabenseifner(x, y) == 0
                ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        want = float(sum(r + 1 + 100 * (k - 1) for r in range(size)))
        exact = bool(torch.all(y == want).item())
        res.append({"buffers": k, "call_us_median": round(statistics.median(ts) * 1e6, 1),
                    "call_us_max": round(max(ts) * 1e6, 1), "calls": len(ts), "exact": exact})
        if rank == 0:
            print(json.dumps(res[-1]), flush=True)
        del xs
    if rank == 0 and out:
        with open(out, "w") as f:
            json.dump({"ranks": size, "count": n, "rows": res}, f, indent=1)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
