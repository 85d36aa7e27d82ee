"""End-to-end (host buffers) Raben timing under ftrun: pinned H2D + device Allreduce +
D2H per call, the chunk pipeline on and off (FTAR_HOST_PIPE is read per job, so this
runs the job twice via the caller).  E2E_ALGO=rd times recursive doubling.  E2E_ZERO_COPY=1 times the device entry point on the
same pinned buffers instead: this rank's kernels read sbuf and write rbuf over PCIe, only
the part peers pull is staged in HBM.

    fault-tolerant_amd/bin/ftrun -np 2 --devmap 0,0 python tools/e2e_probe.py [count]
"""
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    rank = int(os.environ["FTAR_RANK"])
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    comm.set_profiling(os.environ.get("FTAR_PROFILE", "0") == "1")
    xh = (torch.rand(n) * 2 - 1).pin_memory()
    yh = torch.empty_like(xh).pin_memory()
    zc = os.environ.get("E2E_ZERO_COPY", "0") == "1"
    rd = os.environ.get("E2E_ALGO", "raben") == "rd"
    if rd:
        fn = comm.recursive_doubling if zc else comm.recursive_doubling_host
    else:
        fn = comm.allreduce_rabenseifner if zc else comm.allreduce_rabenseifner_host
    for _ in range(2):
        assert fn(xh, yh) == 0
    ts = []
    for _ in range(5):
        comm.barrier()
        t0 = time.perf_counter()
        assert fn(xh, yh) == 0
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    if rank == 0:
        print(json.dumps({"algo": "rd" if rd else "raben", "ranks": int(os.environ["FTAR_SIZE"]), "count": n,
                          "host_pipe": os.environ.get("FTAR_HOST_PIPE", "1"), "zero_copy": zc,
                          "profiling": os.environ.get("FTAR_PROFILE", "0"),
                          "ms_median": round(ts[len(ts) // 2] * 1e3, 3), "ms_min": round(ts[0] * 1e3, 3)}), flush=True)
    comm.finalize()


if __name__ == "__main__":
    main()
