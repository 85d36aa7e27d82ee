"""A / B of the mesh's allgather ordering (FTAR_OPT_MESH_WAIT): ordered on the device behind
the peers' trees (1, the default) or launched after the reduce-scatter's host agree (0), in
one job, interleaved blocks of calls so drift hits both alike; ranks sharing GPU 0.

    fault-tolerant_amd/bin/ftrun -np 4 --devmap 0,0,0,0 python tools/devwait_ab.py [out.json]

Per size (rank 0's clock, each call started right after a barrier): median call time,
median agree-wait and drain-wait per call, peer waits counted.
AB_SIZES (bytes, comma list; default 4 MiB, 64 MiB, 256 MiB), AB_BLOCKS (default 6), AB_CALLS
(calls per block, default 20).
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
    return v[len(v) // 2]


def main():
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    rank, size = int(os.environ["FTAR_RANK"]), int(os.environ["FTAR_SIZE"])
    sizes = [int(s) for s in os.environ.get("AB_SIZES", f"{4 << 20},{64 << 20},{256 << 20}").split(",")]
    blocks, calls = int(os.environ.get("AB_BLOCKS", "6")), int(os.environ.get("AB_CALLS", "20"))
    out = {"ranks": size, "blocks": blocks, "calls_per_block": calls, "sizes": {}}
    comm.set_option(ftar.OPT_ONESHOT_MAX, 0)  # the two-launch mesh at every size (p = 2 too)
    for nbytes in sizes:
        x = torch.rand(nbytes // 4, device="cuda")
        y = torch.empty_like(x)
        res = {w: {"call_us": [], "agree_us": [], "drain_us": [], "peer_waits": 0} for w in (1, 0)}
        for b in range(blocks):
            for w in ((1, 0) if b % 2 == 0 else (0, 1)):
                comm.set_option(ftar.OPT_MESH_WAIT, w)
                comm.allreduce_rabenseifner(x, y)  # warm the form
                for _ in range(calls):
                    comm.barrier()
                    t0 = time.perf_counter()
                    rc = comm.allreduce_rabenseifner(x, y)
                    dt = time.perf_counter() - t0
                    assert rc == 0, rc
                    st = comm.last_stats()
                    res[w]["call_us"].append(dt * 1e6)
                    res[w]["agree_us"].append(st.sync_wait_s * 1e6)
                    res[w]["drain_us"].append(st.drain_s * 1e6)
                    res[w]["peer_waits"] += st.peer_waits
        row = {}
        for w, r in res.items():
            row["device_wait" if w else "host_agree"] = {
                "call_us_median": round(med(r["call_us"]), 1), "agree_wait_us_median": round(med(r["agree_us"]), 1),
                "drain_wait_us_median": round(med(r["drain_us"]), 1), "peer_waits": r["peer_waits"],
                "calls": len(r["call_us"])}
        out["sizes"][str(nbytes)] = row
        del x, y
        torch.cuda.empty_cache()
    comm.set_option(ftar.OPT_MESH_WAIT, 1)
    if rank == 0:
        line = json.dumps(out)
        print(line)
        if len(sys.argv) > 1:
            with open(sys.argv[1], "w") as f:
                f.write(line + "\n")
    comm.finalize()


if __name__ == "__main__":
    main()
