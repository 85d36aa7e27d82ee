"""Per-call time of small (4 KiB) Allreduces, ranks sharing one GPU (ftrun job), under the
conditions that changed it in round 3: gates on / off (EXP_GATES), calls
back to back / barrier-separated / spaced (EXP_MODES), a device synchronize or the latency
probe's prologue before timing (EXP_WARM), bench-like 256 MiB tensors (EXP_BIG), a call
that used the background stream (EXP_BG=1) or a torch side stream used once / only created
(EXP_BG=2 / 3).  Also a torch copy + synchronize as the device round trip without the library.

    EXP_BG=2 fault-tolerant_amd/bin/ftrun -np 2 --devmap 0,0 python tools/small_call_probe.py
"""
import importlib.util, json, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("ftar_amd", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
ftar = importlib.util.module_from_spec(spec); spec.loader.exec_module(ftar)
rank = int(os.environ.get("FTAR_RANK", "0"))
torch.cuda.set_device(0)
comm = ftar.Comm.from_env()
if os.environ.get("EXP_BIG") == "1":  # bench-like: 256 MiB tensors, big calls first (peers read x in place)
    x = torch.rand(1 << 26, device="cuda"); y = torch.empty_like(x)
    for _ in range(10):
        assert comm.allreduce_rabenseifner(x, y) == 0
        assert comm.recursive_doubling(x, y) == 0
else:
    x = torch.rand(1024, device="cuda"); y = torch.empty_like(x)
res = {"ranks": comm.size}
if os.environ.get("EXP_BG") in ("2", "3"):  # an extra torch stream: used once (2) or only created (3)
    side = torch.cuda.Stream()
    if os.environ.get("EXP_BG") == "2":
        with torch.cuda.stream(side):
            y.copy_(x)
        side.synchronize()
if os.environ.get("EXP_BG") == "1":  # a call that uses the background stream (step-0 redundancy copy, overlapped)
    for o, v in ((ftar.OPT_REDUNDANCY, 1), (ftar.OPT_OVERLAP, 1), (ftar.OPT_MESH, 0)):
        comm.set_option(o, v)
    for _ in range(3):
        assert comm.allreduce_rabenseifner(x, y, count=1024) == 0
    for o, v in ((ftar.OPT_REDUNDANCY, 0), (ftar.OPT_MESH, 1)):
        comm.set_option(o, v)
W = os.environ.get("EXP_WARM", "0")
if W == "1":  # the latency probe's prologue: torch copy + synchronize, barriers
    for _ in range(200):
        comm.barrier(); y.copy_(x); torch.cuda.synchronize()
    for _ in range(200):
        comm.barrier()
elif W == "sync1":  # one device synchronize
    torch.cuda.synchronize()
elif W == "copies":  # torch copies + synchronize, no barriers
    for _ in range(200):
        y.copy_(x); torch.cuda.synchronize()
elif W == "barriers":
    for _ in range(400):
        comm.barrier()
if os.environ.get("EXP_MODES"):
    pass
def pct(v, q):
    v = sorted(v); return round(v[int(len(v) * q)] * 1e6, 1)
tt = []
for _ in range(300):
    comm.barrier(); t0 = time.perf_counter(); y.copy_(x); torch.cuda.synchronize(); tt.append(time.perf_counter() - t0)
res["torch_copy_sync"] = {"p50": pct(tt, .5), "p10": pct(tt, .1)}
for gate in [int(g) for g in os.environ.get("EXP_GATES", "1,0").split(",")]:
    comm.set_option(ftar.OPT_GATE, gate)
    for mode in os.environ.get("EXP_MODES", "barrier,b2b,sleep50").split(","):
        for name, fn in (("raben", comm.allreduce_rabenseifner), ("rd", comm.recursive_doubling)):
            for _ in range(10): assert fn(x, y, count=1024) == 0
            comm.barrier()
            wall, dr, sw = [], [], []
            for _ in range(300):
                if mode == "barrier": comm.barrier()
                elif mode == "sleep50":
                    t = time.perf_counter()
                    while time.perf_counter() - t < 50e-6: pass
                t0 = time.perf_counter(); assert fn(x, y, count=1024) == 0; wall.append(time.perf_counter() - t0)
                st = comm.last_stats(); dr.append(st.drain_s); sw.append(st.sync_wait_s)
            res[f"g{gate}_{mode}_{name}"] = {"p10": pct(wall, .1), "p50": pct(wall, .5), "p90": pct(wall, .9),
                                             "drain50": pct(dr, .5), "sync50": pct(sw, .5)}
if rank == 0:
    print(json.dumps(res), flush=True)
comm.finalize()
