"""TEST worker: one rank of a growing-size job under ftrun (tests/test_gpu_schedules.py).

Calls both schedules on int32 vectors of rank ids at sizes 4 KiB .. 256 MiB in one job,
fresh torch allocations at every size: the workspace grows (new exports) while peers
hold mappings of earlier send buffers.  Checks every element against the closed form
sum_r r and writes "ok" / the first failure to $FTAR_PROBE_DIR/grow_<rank>.txt.
"""
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rank, size = int(os.environ["FTAR_RANK"]), int(os.environ["FTAR_SIZE"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    want = size * (size - 1) // 2
    msg = "ok"
    for n in [1 << 10, 1 << 16, 1 << 20, (1 << 22) + 3, 1 << 24, 1 << 26]:
        x = torch.full((n,), rank, dtype=torch.int32, device="cuda")
        for name in ("allreduce_rabenseifner", "recursive_doubling"):
            y = torch.zeros_like(x)
            rc = getattr(comm, name)(x, y)
            torch.cuda.synchronize()
            bad = int((y != want).sum().item())
            if rc != 0 or bad:
                msg = f"{name} n={n} rc={rc} wrong={bad}"
                break
        if msg != "ok":
            break
    # the workspace was re-allocated and re-exported at every growth: every block's IPC
    # export must have succeeded on the first try
    with open(os.path.join(os.environ["FTAR_PROBE_DIR"], f"grow_{rank}.txt"), "w") as f:
        f.write(f"{msg} retries={comm.last_stats().export_retries}")
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
