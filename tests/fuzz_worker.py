"""TEST worker: one rank of a randomized call-sequence job under ftrun (tests/test_gpu_schedules.py).

Every rank draws the same sequence of calls from FTAR_FUZZ_SEED: schedule, dtype, op, length
(0 .. 3 Mi, ragged), element offset into a larger allocation, in place or not, and whether the
send buffer is a fresh allocation or one of the buffers used before (so the peers' mapping
caches see new, repeated and re-allocated buffers, in place and at offsets, between calls of
every size class).  Inputs are small integers from (element, rank, call), so every op's
result -- in every dtype, floats included -- has one exact value, which each rank computes
from all ranks' inputs itself.  Writes "ok <calls>" or the first failure to
$FTAR_PROBE_DIR/fuzz_<rank>.txt.
"""
import importlib.util
import os
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DTYPES = [(torch.int32, 0), (torch.float32, 1), (torch.int64, 2), (torch.float64, 3)]
INT_OPS = list(range(10))
FLOAT_OPS = [0, 1, 2, 3]


def inputs(n, rank, call, dt):
    i = torch.arange(n, device="cuda", dtype=torch.int64)
    return (((i * (rank + 3) + call * 7 + rank) % 7) - 3).to(dt)


def expected(op, xs):
    acc = xs[0].clone()
    for x in xs[1:]:
        if op == 0:
            acc = acc + x
        elif op == 1:
            acc = acc * x
        elif op == 2:
            acc = torch.maximum(acc, x)
        elif op == 3:
            acc = torch.minimum(acc, x)
        elif op == 4:
            acc = ((acc != 0) & (x != 0)).to(acc.dtype)
        elif op == 5:
            acc = acc & x
        elif op == 6:
            acc = ((acc != 0) | (x != 0)).to(acc.dtype)
        elif op == 7:
            acc = acc | x
        elif op == 8:
            acc = ((acc != 0) ^ (x != 0)).to(acc.dtype)
        else:
            acc = acc ^ x
    return acc


def main():
    rank, size = int(os.environ["FTAR_RANK"]), int(os.environ["FTAR_SIZE"])
    ncalls = int(os.environ.get("FTAR_FUZZ_CALLS", "120"))
    rng = random.Random(int(os.environ.get("FTAR_FUZZ_SEED", "1")))
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    pool = []  # (allocation, dtype) of earlier send buffers
    msg = f"ok {ncalls}"
    for call in range(ncalls):
        algo = rng.choice(["allreduce_rabenseifner", "recursive_doubling"])
        dt, code = rng.choice(DTYPES)
        op = rng.choice(INT_OPS if code in (0, 2) else FLOAT_OPS)
        # around every size threshold too: FTAR_STAGE_MAX / FTAR_ONESHOT_MAX / FTAR_GATE_MAX (1 MiB = 2^18
        # 4-byte or 2^17 8-byte elements), the relay's 4 MiB windows
        n = rng.choice([0, 1, 2, 3, 5, 17, 255, 1000, 4099, 65536, 100003, (1 << 17) - 1, 1 << 17, (1 << 17) + 1,
                        (1 << 18) - 1, 1 << 18, (1 << 18) + 1, 1 << 20, (1 << 20) + 9, 3 << 20])
        off = rng.choice([0, 0, 1, 3, 4, 64])
        inplace = rng.random() < 0.3
        fresh = rng.random() < 0.4
        reuse = [b for b in pool if b[1] == dt and b[0].numel() >= off + n]
        if fresh or not reuse:
            base = torch.empty(off + n + rng.choice([0, 5]), dtype=dt, device="cuda")
            pool.append((base, dt))
            if len(pool) > 10:
                pool.pop(0)
        else:
            base = rng.choice(reuse)[0]
        x = base[off:off + n]
        x.copy_(inputs(n, rank, call, dt))
        out = x if inplace else torch.full((n,), -77, dtype=dt, device="cuda")
        torch.cuda.synchronize()
        if n == 0:
            continue  # the reference's count 0 (FTAR_ERR_UNKNOWN) is covered elsewhere
        rc = getattr(comm, algo)(x, out, count=n, dtype=code, op=op)
        torch.cuda.synchronize()
        want = expected(op, [inputs(n, r, call, dt) for r in range(size)])
        bad = int((out != want).sum().item())
        if rc != 0 or bad:
            msg = f"call {call}: {algo} dtype {code} op {op} n {n} off {off} inplace {inplace} fresh {fresh}: rc {rc} wrong {bad}"
            break
    with open(os.path.join(os.environ["FTAR_PROBE_DIR"], f"fuzz_{rank}.txt"), "w") as f:
        f.write(msg)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
