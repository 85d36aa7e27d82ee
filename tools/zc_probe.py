"""Host-resident local reduce on one GPU, three ways (end-to-end rate):

  serial     pinned H2D of both vectors, the kernel, pinned D2H of the result (bench.py e2e)
  zero_copy  the kernel reads both vectors straight from pinned host memory over PCIe and
             writes the result back into host memory: reads and writes share the link's
             two directions instead of taking turns
  pipeline   the serial form in chunks on three streams (H2D / kernel / D2H)

Every form is checked element for element against a CPU sum.  Prints one JSON line.
    python tools/zc_probe.py [count] [iters]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import importlib.util
    spec = importlib.util.spec_from_file_location("ftar", os.path.join(ROOT, "fault-tolerant_amd", "__init__.py"))
    ftar = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ftar)
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    variant = int(os.environ.get("ZC_VARIANT", "0"))
    torch.cuda.set_device(0)
    S = count * 4
    g = torch.Generator().manual_seed(3)
    x0 = torch.rand(count, generator=g)
    y0 = torch.rand(count, generator=g)
    want = x0 + y0
    xh = x0.pin_memory()
    yh = torch.empty(count).pin_memory()
    xd = torch.empty(count, device="cuda")
    yd = torch.empty(count, device="cuda")
    st = torch.cuda.current_stream()
    out = {"count": count, "bytes_per_vector": S, "iters": iters, "kernel_variant": variant}

    def check(name):
        ok = torch.equal(yh, want)
        out[name]["exact"] = bool(ok)
        return ok

    # serial
    ftar.set_reduce_variant(1)
    ts = []
    for _ in range(iters):
        yh.copy_(y0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        xd.copy_(xh, non_blocking=True)
        yd.copy_(yh, non_blocking=True)
        ftar.reduce_local(xd, yd)
        yh.copy_(yd, non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    out["serial"] = {"ms": round(t * 1e3, 3), "GBps": round(2 * S / t / 1e9, 2)}
    check("serial")

    # zero copy: host pointers straight into the kernel
    ftar.set_reduce_variant(variant)
    ts = []
    for _ in range(iters):
        yh.copy_(y0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ftar.reduce_local(xh.data_ptr(), yh.data_ptr(), count=count, dtype=ftar.FLOAT32, stream=st.cuda_stream)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    out["zero_copy"] = {"ms": round(t * 1e3, 3), "GBps": round(2 * S / t / 1e9, 2),
                        "pcie_GBps": round(3 * S / t / 1e9, 2)}
    check("zero_copy")

    # chunk pipeline on three streams
    ftar.set_reduce_variant(1)
    nch = int(os.environ.get("ZC_CHUNKS", "16"))
    per = (count + nch - 1) // nch
    s_h2d, s_k, s_d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    ts = []
    for _ in range(iters):
        yh.copy_(y0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev_in, ev_k = [], []
        for c in range(nch):
            a, b = c * per, min(count, (c + 1) * per)
            with torch.cuda.stream(s_h2d):
                xd[a:b].copy_(xh[a:b], non_blocking=True)
                yd[a:b].copy_(yh[a:b], non_blocking=True)
                e = torch.cuda.Event()
                e.record(s_h2d)
            s_k.wait_event(e)
            ftar.reduce_local(xd[a:b], yd[a:b], stream=s_k.cuda_stream)
            e2 = torch.cuda.Event()
            e2.record(s_k)
            s_d2h.wait_event(e2)
            with torch.cuda.stream(s_d2h):
                yh[a:b].copy_(yd[a:b], non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    out["pipeline"] = {"ms": round(t * 1e3, 3), "GBps": round(2 * S / t / 1e9, 2), "chunks": nch}
    check("pipeline")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
