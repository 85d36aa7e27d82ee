"""GPU parity of the local-reduce kernel (MPI_Reduce_local) against the CPU oracle.

Bar: bit-exact for every dtype/op on the same inputs (one IEEE op per element for
floats; two's-complement wrap for ints).  Sizes cover empty, ragged, unaligned heads
and tails, non-co-aligned pointers (scalar path) and the full 256 MiB C2 vector.
"""
import os
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NP = {0: np.int32, 1: np.float32, 2: np.int64, 3: np.float64}
UINT = {4: np.uint32, 8: np.uint64}


def _inputs(dt, n, seed, specials=False):
    rng = np.random.default_rng(seed)
    t = NP[dt]
    if np.dtype(t).kind == "f":
        a = (rng.standard_normal(n) * 100).astype(t)
        b = (rng.standard_normal(n) * 100).astype(t)
        if specials and n >= 16:
            sp = np.array([0.0, -0.0, np.inf, -np.inf, 1e-40, -1e-40, 3.4e38, -3.4e38], dtype=t)
            a[:8] = sp
            b[8:16] = sp
    else:
        info = np.iinfo(t)
        a = rng.integers(info.min, info.max, n, dtype=t, endpoint=True)
        b = rng.integers(info.min, info.max, n, dtype=t, endpoint=True)
    return a, b


def _same_bits(x, y):
    u = UINT[x.dtype.itemsize]
    return np.array_equal(x.view(u), y.view(u))


def _to_dev(a):
    import torch
    return torch.from_numpy(a.copy()).cuda()


@pytest.mark.parametrize("dt", [0, 1, 2, 3])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [0, 1, 3, 17, 1000, 65537, 1 << 20])
def test_reduce_local_bit_exact(ftar, oracle, dt, op, n):
    import torch
    a, b = _inputs(dt, n, seed=n * 7 + op, specials=(op >= 2 or n > 100))
    x, y = _to_dev(a), _to_dev(b)
    ftar.reduce_local(x, y, op=op)  # y = y <op> x
    torch.cuda.synchronize()
    want = b.copy()
    oracle.reduce_local(a, want, op)
    assert _same_bits(y.cpu().numpy(), want)


@pytest.mark.parametrize("off_in,off_io", [(1, 1), (3, 3), (1, 2), (0, 3), (2, 0)])
def test_reduce_local_unaligned(ftar, oracle, off_in, off_io):
    """Heads/tails (co-aligned offsets) and the scalar path (different alignments)."""
    import torch
    n = 100003
    a, b = _inputs(1, n + 8, seed=11)
    x, y = _to_dev(a), _to_dev(b)
    ftar.reduce_local(x[off_in:off_in + n], y[off_io:off_io + n], count=n, dtype=1, op=0)
    torch.cuda.synchronize()
    want = b.copy()
    part = want[off_io:off_io + n].copy()
    oracle.reduce_local(a[off_in:off_in + n].copy(), part, 0)
    want[off_io:off_io + n] = part
    assert _same_bits(y.cpu().numpy(), want)  # untouched outside the window too


@pytest.mark.parametrize("variant", [0, 1])
def test_reduce_local_c2_full_size(ftar, variant):
    """C2: two 256 MiB float32 vectors; property check against torch's own fp32 add
    (one IEEE add per element, so bit-identical)."""
    import torch
    n = 1 << 26
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y = torch.rand(n, device="cuda", generator=g) * 2 - 1
    want = y + x
    ftar.set_reduce_variant(variant)
    try:
        ftar.reduce_local(x, y, op=0)
        torch.cuda.synchronize()
    finally:
        ftar.set_reduce_variant(0)
    assert torch.equal(y.view(torch.int32), want.view(torch.int32))


@pytest.mark.parametrize("variant,extra", [(0, 4099), (1, 4100)])
def test_reduce_local_beyond_2g_elements(ftar, variant, extra):
    """More than 2^31 elements (8 GiB per vector): 64-bit indexing in both kernels and
    the capped, grid-stride launch; a ragged tail for the register kernel.  Checked
    against torch's fp32 add (one IEEE add per element, so bit-identical)."""
    import torch
    n = (1 << 31) + extra
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.rand(n, device="cuda", generator=g)
    y = torch.rand(n, device="cuda", generator=g)
    want = y + x
    ftar.set_reduce_variant(variant)
    try:
        ftar.reduce_local(x, y, op=0)
        torch.cuda.synchronize()
    finally:
        ftar.set_reduce_variant(0)
    assert torch.equal(y.view(torch.int32), want.view(torch.int32))
    del x, y, want
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dt", [0, 1, 2, 3])
def test_reduce_local_lds_variant_bit_exact(ftar, oracle, dt):
    import torch
    n = (1 << 20) + 256  # multiple of 16 bytes for every dtype
    a, b = _inputs(dt, n, seed=dt)
    x, y = _to_dev(a), _to_dev(b)
    ftar.set_reduce_variant(1)
    try:
        ftar.reduce_local(x, y, op=0)
        torch.cuda.synchronize()
    finally:
        ftar.set_reduce_variant(0)
    want = b.copy()
    oracle.reduce_local(a, want, 0)
    assert _same_bits(y.cpu().numpy(), want)


def test_reduce_local_rejects_bad_args(ftar):
    import torch
    x = torch.zeros(16, device="cuda")
    with pytest.raises(ftar.FtarError):
        ftar.reduce_local(x, x, dtype=9)


@pytest.mark.parametrize("dt", [0, 2])
@pytest.mark.parametrize("op", [4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("n", [1, 17, 65537, 1 << 20])
def test_reduce_local_logical_bitwise(ftar, oracle, dt, op, n):
    """MPI's logical / bitwise ops on the integer types: vector body, heads and tails
    bit-exact to the oracle; inputs carry zeros for the logical ops."""
    import torch
    a, b = _inputs(dt, n, seed=n * 3 + op)
    a[::3] = 0
    b[1::5] = 0
    x, y = _to_dev(a), _to_dev(b)
    ftar.reduce_local(x, y, op=op)
    torch.cuda.synchronize()
    want = b.copy()
    oracle.reduce_local(a, want, op)
    assert _same_bits(y.cpu().numpy(), want)


@pytest.mark.parametrize("dt", [1, 3])
def test_reduce_local_bitwise_on_float_refused(ftar, dt):
    """MPI_ERR_OP before any launch; the output is untouched."""
    import torch
    x = torch.ones(1000, device="cuda", dtype=torch.float32 if dt == 1 else torch.float64)
    y = torch.full_like(x, 2.0)
    for op in range(4, 10):
        with pytest.raises(ftar.FtarError, match="code 9"):
            ftar.reduce_local(x, y, op=op)
    torch.cuda.synchronize()
    assert bool((y == 2.0).all())


def _pinned(a):
    import torch
    return torch.from_numpy(a.copy()).pin_memory()


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("dt", [0, 1, 2, 3])
@pytest.mark.parametrize("op", [0, 2, 3])
@pytest.mark.parametrize("n", [1, 17, 65537, (1 << 20) + 256])
def test_reduce_local_pinned_host(ftar, oracle, variant, dt, op, n):
    """The reference's MPI_Reduce_local works on host buffers: with pinned ones the kernel
    reads and writes them in place over PCIe (zero copy).  Bit-exact to the oracle, both
    kernels, the vector body and the scalar heads / tails."""
    import torch
    a, b = _inputs(dt, n, seed=n * 5 + op + dt, specials=op >= 2)
    x, y = _pinned(a), _pinned(b)
    ftar.set_reduce_variant(variant)
    try:
        ftar.reduce_local(x, y, op=op)
        torch.cuda.synchronize()
    finally:
        ftar.set_reduce_variant(0)
    want = b.copy()
    oracle.reduce_local(a, want, op)
    assert _same_bits(y.numpy(), want)


@pytest.mark.parametrize("where", ["in_host", "inout_host"])
def test_reduce_local_mixed_host_device(ftar, oracle, where):
    """One operand in pinned host memory, the other in HBM."""
    import torch
    n = 300007
    a, b = _inputs(1, n, seed=23)
    x = _pinned(a) if where == "in_host" else _to_dev(a)
    y = _pinned(b) if where == "inout_host" else _to_dev(b)
    ftar.reduce_local(x, y, op=0)
    torch.cuda.synchronize()
    want = b.copy()
    oracle.reduce_local(a, want, 0)
    assert _same_bits(y.cpu().numpy(), want)


@pytest.mark.parametrize("off_in,off_io", [(1, 1), (1, 2)])
def test_reduce_local_pinned_unaligned(ftar, oracle, off_in, off_io):
    import torch
    n = 100003
    a, b = _inputs(1, n + 8, seed=29)
    x, y = _pinned(a), _pinned(b)
    ftar.reduce_local(x[off_in:off_in + n], y[off_io:off_io + n], count=n, dtype=1, op=0)
    torch.cuda.synchronize()
    want = b.copy()
    part = want[off_io:off_io + n].copy()
    oracle.reduce_local(a[off_in:off_in + n].copy(), part, 0)
    want[off_io:off_io + n] = part
    assert _same_bits(y.numpy(), want)


def test_reduce_local_c2_pinned_host_full_size(ftar):
    """C2's two 256 MiB float32 vectors in pinned host memory, reduced in place over PCIe
    (bench.py's e2e.zero_copy); checked against torch's fp32 add on the CPU (one IEEE add
    per element, so bit-identical)."""
    import torch
    n = 1 << 26
    g = torch.Generator().manual_seed(13)
    x = (torch.rand(n, generator=g) * 2 - 1).pin_memory()
    y = (torch.rand(n, generator=g) * 2 - 1).pin_memory()
    want = y + x
    ftar.set_reduce_variant(1)
    try:
        ftar.reduce_local(x, y, op=0)
        torch.cuda.synchronize()
    finally:
        ftar.set_reduce_variant(0)
    assert torch.equal(y.view(torch.int32), want.view(torch.int32))


def test_reduce_local_refuses_pageable_and_overruns(ftar):
    """Pageable host memory (a kernel touching it would fault the GPU) and a range past
    its device allocation are refused with FTAR_ERR_ARG before any launch."""
    import torch
    page = np.arange(4096, dtype=np.float32)
    y = torch.full((4096,), 2.0, device="cuda")
    with pytest.raises(ftar.FtarError, match="code 13"):
        ftar.reduce_local(page.ctypes.data, y, count=4096, dtype=1)
    with pytest.raises(ftar.FtarError, match="code 13"):
        ftar.reduce_local(y, page.ctypes.data, count=4096, dtype=1)
    with pytest.raises(ftar.FtarError):
        ftar.reduce_local(torch.from_numpy(page), y)  # not pinned: refused in the binding
    x = torch.ones(16, device="cuda")
    with pytest.raises(ftar.FtarError, match="code 13"):
        ftar.reduce_local(x, y, count=1 << 30, dtype=1)
    torch.cuda.synchronize()
    assert bool((y == 2.0).all())
    assert np.array_equal(page, np.arange(4096, dtype=np.float32))


def test_short_pinned_buffers_refused(ftar):
    """A pinned host buffer shorter than `count`: refused with FTAR_ERR_ARG by the
    local reduce and by both Allreduce entry points before anything is launched -- the GPU
    would otherwise page-fault past the pinned allocation."""
    import torch
    short = torch.ones(1024).pin_memory()
    y = torch.full((1 << 20,), 2.0).pin_memory()
    yd = torch.full((1 << 20,), 2.0, device="cuda")
    for a, b in ((short, yd), (yd, short), (short, y)):
        with pytest.raises(ftar.FtarError, match="code 13"):
            ftar.reduce_local(a, b, count=1 << 20, dtype=1)
    comm = ftar.Comm.init_rank(f"/ftar-pin-{os.getpid()}", 0, 1, 0)
    try:
        assert comm.allreduce_rabenseifner(short, yd, count=1 << 20) == ftar.ERR_ARG
        assert comm.allreduce_rabenseifner(yd, short, count=1 << 20) == ftar.ERR_ARG
        assert comm.recursive_doubling(short, yd, count=1 << 20) == ftar.ERR_ARG
        assert comm.recursive_doubling(yd, short, count=1 << 20) == ftar.ERR_ARG
        # the same buffers at their own length go through (zero copy on pinned memory)
        assert comm.allreduce_rabenseifner(short, short, count=1024) == 0
    finally:
        comm.finalize()
    torch.cuda.synchronize()
    assert bool((yd == 2.0).all()) and bool((y == 2.0).all()) and bool((short == 1.0).all())


@pytest.mark.timeout(300)
def test_tree_kernels_against_oracle():
    """The mesh's tree kernels on their own (tests/kernel_gpu/tree_check.hip, built by
    __graft_entry__.build()): tree_kernel at p = 2, 4, 8 AND 16 (the schedules reach p = 16
    only with 16 ranks), unroll 1 / 2 / 4, extra destinations (push2), co-aligned and
    mutually misaligned pointers, ragged lengths up to 2^20 + 7, and tree_batch_kernel (the
    one-shot form, 1 / 3 / 8 trees), float32 / float64 / int32 / int64 with SUM, PROD, MAX,
    MIN and MPI's logical / bitwise ops -- bit-exact against the balanced tree computed by
    the oracle's reduce_local, MAX / MIN over NaN, signed zeros and infinities."""
    _run_checker("tree_check")


def _run_checker(name, *args):
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "kernel_gpu", "_build",
                       name)
    assert os.path.exists(exe), "tests/kernel_gpu not built: run __graft_entry__.build()"
    cp = subprocess.run([exe, *args], capture_output=True, text=True, timeout=280)
    assert cp.returncode == 0, (cp.stdout[-3000:], cp.stderr[-2000:])
    assert " 0 failed" in cp.stdout, cp.stdout[-3000:]


@pytest.mark.timeout(300)
def test_segment_kernel_against_oracle():
    """The segment kernel on its own (tests/kernel_gpu/seg_check.hip): 400 random lists of
    up to 16 copy / reduce pieces as the schedules build them -- ragged lengths up to 2^20,
    co-aligned and misaligned pointers, a second destination holding the result or (the
    mid-exchange guard) the local operand's pre-image, grids capped at 2^20 / 1024 / 128 / 7
    workgroups -- bit-exact against the oracle, nothing written outside a destination,
    sources untouched; MAX / MIN over NaN, signed zeros and infinities."""
    _run_checker("seg_check")
