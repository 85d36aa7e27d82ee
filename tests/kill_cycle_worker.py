"""TEST worker: one rank of a send-buffer cycling job with a rank killed mid-job (FTAR_KILL,
set by tests/test_gpu_schedules.py), recursive doubling (which recovers at any p).

Cycles 9 device buffers (more than the peers' mapping caches hold; buffer i holds
rank + 1 + 100 i) through 24 calls.  Per call it records rc, the comm size after the call,
the result's first element and whether every element equals it, in
$FTAR_PROBE_DIR/kc_<rank>.json: calls before the kill must sum every rank, calls after it the survivors.
"""
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rank = int(os.environ["FTAR_RANK"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    n, k = 1 << 22, 9
    xs = [torch.full((n,), float(rank + 1 + 100 * i), device="cuda") for i in range(k)]
    y = torch.empty(n, device="cuda")
    calls = []
    for c in range(24):
        i = c % k
        rc = comm.recursive_doubling(xs[i], y)
        torch.cuda.synchronize()
        v = float(y[0].item())
        calls.append({"buffer": i, "rc": rc, "size": comm.size, "value": v, "uniform": bool((y == v).all().item())})
    with open(os.path.join(os.environ["FTAR_PROBE_DIR"], f"kc_{rank}.json"), "w") as f:
        json.dump({"rank": rank, "calls": calls}, f)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
