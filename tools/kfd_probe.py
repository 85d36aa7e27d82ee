#!/usr/bin/env python3
"""Which step of a bench rank first opens the GPU driver (/dev/kfd, /dev/dri/render*)?

bench.py's N > 1 ranks wait for rank 0's side legs (CPU baseline, the 9-rank configs[4]
jobs, the fabric probe) before importing torch, so that the job's own ranks are not GPU
processes while those legs run.  This prints, after each stage, the GPU device files the
process holds open and whether KFD lists it (/sys/class/kfd/kfd/proc/<pid>).
"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def held():
    fds = []
    for fd in os.listdir("/proc/self/fd"):
        try:
            t = os.readlink(f"/proc/self/fd/{fd}")
        except OSError:
            continue
        if t.startswith("/dev/kfd") or t.startswith("/dev/dri"):
            fds.append(t)
    return {"fds": sorted(set(fds)), "kfd_proc": os.path.exists(f"/sys/class/kfd/kfd/proc/{os.getpid()}")}


out = {"start": held()}
import torch  # noqa: E402

out["import_torch"] = held()
n = torch.cuda.device_count()
out["device_count"] = dict(held(), n=n)
spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
mod = importlib.util.module_from_spec(spec)
sys.modules["ftar_amd"] = mod
spec.loader.exec_module(mod)
mod.lib()
out["load_libftar"] = held()
torch.cuda.set_device(0)
x = torch.zeros(16, device="cuda")
out["first_tensor"] = held()
print(json.dumps(out))
