"""TEST worker: one rank of a send-buffer cycling job under ftrun (tests/test_gpu_schedules.py).

A bucketed all-reduce: the caller cycles its send buffer through K distinct allocations
(16 MiB each, FTAR_CYCLE_BUFFERS, default 9 -- more than the peers' mapping cache holds),
three passes, both schedules; FTAR_CYCLE_SLICES=1: the k buffers are views of one allocation
at different offsets (one cache entry, read in place at each view's offset);
FTAR_CYCLE_INPLACE=1: every call in place (the send buffer is the receive buffer).  Each
buffer holds rank + 1 + 100 * i, so every result has a closed form; writes "ok" / the first failure and the median call time to
$FTAR_PROBE_DIR/cycle_<rank>.txt.
"""
import importlib.util
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rank, size = int(os.environ["FTAR_RANK"]), int(os.environ["FTAR_SIZE"])
    k = int(os.environ.get("FTAR_CYCLE_BUFFERS", "9"))
    inplace = os.environ.get("FTAR_CYCLE_INPLACE") == "1"
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    n = 1 << 22
    if os.environ.get("FTAR_CYCLE_SLICES") == "1":  # k views of ONE allocation: one id, k offsets
        big = torch.empty(k * n + 5, device="cuda")
        xs = [big[5 + i * n:5 + (i + 1) * n] for i in range(k)]
        for i, x in enumerate(xs):
            x.fill_(float(rank + 1 + 100 * i))
    else:
        xs = [torch.full((n,), float(rank + 1 + 100 * i), device="cuda") for i in range(k)]
    y = torch.empty(n, device="cuda")
    msg, ts = "ok", []
    for name in ("allreduce_rabenseifner", "recursive_doubling"):
        for _ in range(3):
            for i, x in enumerate(xs):
                if inplace:
                    x.fill_(float(rank + 1 + 100 * i))
                    torch.cuda.synchronize()
                out = x if inplace else y
                comm.barrier()
                t0 = time.perf_counter()
                rc = getattr(comm, name)(x, out)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                want = float(sum(r + 1 + 100 * i for r in range(size)))
                bad = int((out != want).sum().item())
                if rc != 0 or bad:
                    msg = f"{name} buffer {i} rc={rc} wrong={bad}"
                    break
            if msg != "ok":
                break
        if msg != "ok":
            break
    with open(os.path.join(os.environ["FTAR_PROBE_DIR"], f"cycle_{rank}.txt"), "w") as f:
        f.write(f"{msg} median_us={statistics.median(ts) * 1e6:.1f}")
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
