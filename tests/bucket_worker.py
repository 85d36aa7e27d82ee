"""TEST worker: one rank of a mixed-bucket job under ftrun (tests/test_gpu_schedules.py).

What a training step's gradient all-reduce looks like to the library: buckets of different
sizes (7 elements .. 6 Mi), dtypes (float32, int32, float64, int64) and both schedules,
interleaved, each bucket its own buffer, the whole step repeated; some buckets in place.
Values are small integers, so every sum has a closed form in every dtype.  Writes "ok" / the
first failure to $FTAR_PROBE_DIR/bucket_<rank>.txt.
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
    dts = [torch.float32, torch.int32, torch.float64, torch.int64]
    sizes = [7, 1000, 65536 + 3, 1 << 18, (1 << 20) + 17, 3 << 20, 6 << 20, 31]
    buckets = []
    for i, n in enumerate(sizes):
        dt = dts[i % len(dts)]
        x = torch.full((n,), rank + 1 + i, dtype=dt, device="cuda")
        buckets.append((i, dt, x, torch.empty_like(x), i % 3 == 2))
    msg = "ok"
    for step in range(4):
        for i, dt, x, y, inplace in (buckets if step % 2 == 0 else buckets[::-1]):
            name = "allreduce_rabenseifner" if (i + step) % 2 == 0 else "recursive_doubling"
            if inplace:
                x.fill_(rank + 1 + i)
            out = x if inplace else y
            rc = getattr(comm, name)(x, out)
            torch.cuda.synchronize()
            want = sum(r + 1 + i for r in range(size))
            bad = int((out != want).sum().item())
            if rc != 0 or bad:
                msg = f"step {step} bucket {i} ({dt}, n={x.numel()}, {name}, inplace={inplace}) rc={rc} wrong={bad}"
                break
        if msg != "ok":
            break
    with open(os.path.join(os.environ["FTAR_PROBE_DIR"], f"bucket_{rank}.txt"), "w") as f:
        f.write(msg)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
