"""Resource soak of one rank: thousands of device-resident Allreduces as a long training job
issues them -- buckets cycled through more send buffers than the peers' mapping caches hold,
and every 100 calls two buckets re-allocated (freed, torch's cache emptied, so the new ones
are new allocations: new exports, new peer mappings, idle evictions of the old) -- sampling
this process's open file descriptors, resident memory and free device memory.

    fault-tolerant_amd/bin/ftrun -np 4 --devmap 0,0,0,0 python tools/leak_soak.py [calls] [out.json]

Rank 0 writes the samples and the growth between the first sample (after warm-up) and the
last; every result is checked (closed-form sums).
"""
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fds():
    return len(os.listdir("/proc/self/fd"))


def rss_mib():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return -1.0


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    out = sys.argv[2] if len(sys.argv) > 2 else None
    rank, size = int(os.environ["FTAR_RANK"]), int(os.environ["FTAR_SIZE"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    n = 1 << 20  # 4 MiB float32 per bucket
    k = 12
    xs = [torch.full((n,), float(rank + 1 + i), device="cuda") for i in range(k)]
    y = torch.empty(n, device="cuda")
    samples, bad, realloc = [], 0, 0
    warm = 200
    for c in range(calls):
        i = c % k
        fn = comm.allreduce_rabenseifner if (c // k) % 2 == 0 else comm.recursive_doubling
        rc = fn(xs[i], y)
        if rc != 0:
            bad += 1
        if c % 50 == 0:
            torch.cuda.synchronize()
            if float(y[0].item()) != float(sum(r + 1 + i for r in range(size))) or float(y[-1].item()) != float(
                    sum(r + 1 + i for r in range(size))):
                bad += 1
        if c % 100 == 99:  # two buckets re-allocated: new allocations, new exports
            torch.cuda.synchronize()
            for j in ((c // 100) % k, (c // 100 + 5) % k):
                xs[j] = None
            torch.cuda.empty_cache()
            for j in ((c // 100) % k, (c // 100 + 5) % k):
                xs[j] = torch.full((n,), float(rank + 1 + j), device="cuda")
            realloc += 2
        if c == warm or c == calls - 1 or (c > warm and c % 500 == 0):
            torch.cuda.synchronize()
            free, total = torch.cuda.mem_get_info()
            samples.append({"call": c, "fds": fds(), "rss_mib": round(rss_mib(), 1),
                            "device_free_gib": round(free / (1 << 30), 3)})
    torch.cuda.synchronize()
    res = {"ranks": size, "calls": calls, "buffers": k, "reallocations": realloc, "bad": bad, "samples": samples,
           "growth_after_warmup": {key: round(samples[-1][key] - samples[0][key], 3)
                                   for key in ("fds", "rss_mib", "device_free_gib")}}
    if rank == 0:
        print(json.dumps(res), flush=True)
        if out:
            with open(out, "w") as f:
                json.dump(res, f, indent=1)
    comm.finalize()
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
