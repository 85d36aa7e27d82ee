"""TEST worker: one rank of a recursive-doubling job whose callers cycle 9 device send buffers
through 3000 calls while the test SIGKILLs a random rank from outside (no injection point:
any instant of the call loop).  Writes $FTAR_PROBE_DIR/ready_<rank> when the loop starts, and
per call the comm size and the result's first element (and whether every element equals it)
to $FTAR_PROBE_DIR/xk_<rank>.txt, one line per call, flushed as it goes.
"""
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rank = int(os.environ["FTAR_RANK"])
    d = os.environ["FTAR_PROBE_DIR"]
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    n, k = 1 << 21, 9
    xs = [torch.full((n,), float(rank + 1 + 100 * i), device="cuda") for i in range(k)]
    y = torch.empty(n, device="cuda")
    comm.barrier()
    open(os.path.join(d, f"ready_{rank}"), "w").close()
    with open(os.path.join(d, f"xk_{rank}.txt"), "w", buffering=1) as f:
        for c in range(3000):
            i = c % k
            rc = comm.recursive_doubling(xs[i], y)
            torch.cuda.synchronize()
            v = float(y[0].item())
            f.write(f"{c} {i} {rc} {comm.size} {v} {int(bool((y == v).all().item()))}\n")
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
