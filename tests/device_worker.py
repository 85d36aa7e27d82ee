"""TEST worker: one rank of a device-buffer parity run, launched by ftrun.

Binds the product library through the package (as bench.py does), puts this rank's
input in a torch tensor on the rank's GPU (optionally at an element offset, optionally
in place: sbuf == rbuf), calls the device-pointer entry point twice and writes the
results plus "rc sbuf_untouched" per call for tests/harness.run_torch_worker.

env: FTAR_PROBE_DIR, FTAR_PROBE_ALGO=rd|raben, FTAR_PROBE_INPLACE, FTAR_PROBE_OFFSET,
FTAR_PROBE_PINNED=1 (sbuf and rbuf in pinned host memory: the kernels read and write them
in place over PCIe, peers read the staged copy),
FTAR_PROBE_REALLOC=1 (the second call gets a freshly allocated sbuf holding -input, after
the first one's memory went back to the driver: a re-used address must not be read
through a stale peer mapping) (set by the harness), FTAR_RANK / FTAR_DEVICE (set by ftrun)
"""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = os.environ["FTAR_PROBE_DIR"]
    algo = os.environ["FTAR_PROBE_ALGO"]
    rank = int(os.environ["FTAR_RANK"])
    inplace = int(os.environ.get("FTAR_PROBE_INPLACE", "0"))
    off = int(os.environ.get("FTAR_PROBE_OFFSET", "0"))
    realloc = int(os.environ.get("FTAR_PROBE_REALLOC", "0"))
    pinned = int(os.environ.get("FTAR_PROBE_PINNED", "0"))
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    a = np.fromfile(os.path.join(d, f"in_{rank}.bin"), dtype=np.float32)
    n = a.size
    want_in = torch.from_numpy(a)

    def buf(fill):
        if pinned:
            return torch.full((n + off + 16,), fill).pin_memory()[off:off + n]
        return torch.full((n + off + 16,), fill, device="cuda")[off:off + n]

    src = buf(0.0)
    for it in range(2):
        if realloc and it:
            del src
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            want_in = -want_in
            src = buf(0.0)
        src.copy_(want_in)
        dst = src if inplace else buf(float("nan"))
        fn = comm.allreduce_rabenseifner if algo == "raben" else comm.recursive_doubling
        rc = fn(src, dst)
        torch.cuda.synchronize()
        untouched = inplace or bool(torch.equal(src.cpu(), want_in))
        dst.cpu().numpy().tofile(os.path.join(d, f"out_{rank}_{it}.bin"))
        with open(os.path.join(d, f"status_{rank}_{it}.txt"), "w") as f:
            f.write(f"{rc} {int(untouched)}\n")
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
