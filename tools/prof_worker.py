"""One rank of a profiling job: `iters` device-resident Allreduces of `count` float32 per
rank with the library's default transport (the mesh at power-of-two p), so rocprofv3
(tools/rank_prof.sh) sees the exchange kernels of the N > 1 bench line -- the tree kernel
and the allgather pulls -- with every rank on one GPU.

    ftrun -np 8 --devmap 0,0,0,0,0,0,0,0 tools/rank_prof.sh OUT trace python3 tools/prof_worker.py [count] [iters] [algo]
"""
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    algo = sys.argv[3] if len(sys.argv) > 3 else "raben"
    torch.cuda.set_device(int(os.environ.get("FTAR_DEVICE", "0")))
    spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    comm = ftar.Comm.from_env()
    x = torch.rand(count, device="cuda") * 2 - 1
    y = torch.empty_like(x)
    fn = comm.allreduce_rabenseifner if algo == "raben" else comm.recursive_doubling
    for _ in range(iters + 3):
        assert fn(x, y) == 0
    torch.cuda.synchronize()
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
