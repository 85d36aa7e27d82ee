"""Python mirror of the reference's Allreduce interface over libftar.so (ctypes).

The product is the C ABI in include/ftar.h (lib/libftar.so: host-C schedules + HIP
kernels for gfx950).  This module only binds it for Python callers (bench.py, the
GPU tests): it keeps the reference's names and argument meaning

    recursive_doubling(src, dst, count, dtype, op)        src/rd/header.h:29
    allreduce_rabenseifner(sbuf, rbuf, count, dtype, op)  src/raben/header.h:14-15
    reduce_local(in, inout, count, dtype, op)             MPI_Reduce_local call sites

and raises if the native library is missing -- there is no Python or CPU fallback.
Buffers are device pointers: ints, or torch tensors on the rank's GPU.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libftar.so")

INT32, FLOAT32, INT64, FLOAT64 = 0, 1, 2, 3
SUM, PROD, MAX, MIN = 0, 1, 2, 3
LAND, BAND, LOR, BOR, LXOR, BXOR = 4, 5, 6, 7, 8, 9  # MPI logical / bitwise ops (integer types)
PH_PRE, PH_LOOP, PH_AG, PH_POST = 0, 1, 2, 3
PT_BEFORE, PT_AFTER, PT_BARRIER, PT_DURING = 0, 1, 2, 3
OPT_OVERLAP, OPT_RELAY, OPT_RELAY_MIN, OPT_LOOP_SECONDS, OPT_COPY_ENGINE, OPT_REDUNDANCY, OPT_MESH = 0, 1, 2, 3, 4, 5, 6
OPT_ONESHOT_MAX = 7
OPT_PUSH = 8
OPT_GATE = 9
OPT_FLAG_SYNC = 10
OPT_TREE_UNROLL = 11
OPT_GATE_MAX = 12
OPT_MESH_WAIT = 13
REDUNDANCY_NEVER, REDUNDANCY_ALWAYS, REDUNDANCY_AUTO = 0, 1, 2  # OPT_REDUNDANCY values
SUCCESS, ERR_ARG, ERR_UNKNOWN, ERR_OTHER, ERR_PROC_FAILED = 0, 13, 14, 16, 75
ERR_OP = 9  # MPI_ERR_OP: a logical / bitwise op on a float type


class FtarError(RuntimeError):
    pass


class Stats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_int), ("recoveries", ctypes.c_int), ("comm_size_after", ctypes.c_int),
                ("wall_s", ctypes.c_double), ("kernel_ms", ctypes.c_double),
                ("step0_kernel_ms", ctypes.c_double), ("link_bytes", ctypes.c_double),
                ("hbm_bytes", ctypes.c_double), ("kernels", ctypes.c_int), ("step0_link_bytes", ctypes.c_double),
                ("bg_kernel_ms", ctypes.c_double), ("sync_wait_s", ctypes.c_double),
                ("drain_s", ctypes.c_double), ("syncs", ctypes.c_int), ("relayed_steps", ctypes.c_int),
                ("mesh_steps", ctypes.c_int), ("export_retries", ctypes.c_int),
                ("gated_launches", ctypes.c_int), ("gated_skips", ctypes.c_int),
                ("user_stream_waits", ctypes.c_int), ("step0_copy", ctypes.c_int), ("gate_holds", ctypes.c_int),
                ("gate_relaunches", ctypes.c_int), ("peer_waits", ctypes.c_int), ("peer_wait_skips", ctypes.c_int)]


class Kill(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int), ("phase", ctypes.c_int), ("step", ctypes.c_int),
                ("point", ctypes.c_int)]


_lib = None
_test_lib_path = None


def use_test_library(path: str):
    """TEST-ONLY: bind the host-memory build of the same C sources (tests/hostsim/_build/
    libftar_hostsim.so) instead of lib/libftar.so, so bench.py's N > 1 control flow can be
    exercised on a CPU-only machine (tests/test_bench_logic.py, `bench.py --device cpu`
    under FTAR_BENCH_CPU_TEST=1).  Refuses any other library, and refuses once the product
    library is bound; the product path and the GPU tests never call it."""
    global _test_lib_path
    if _lib is not None:
        raise FtarError("the product library is already bound")
    if os.path.basename(path) != "libftar_hostsim.so" or not os.path.exists(path):
        raise FtarError(f"{path} is not the host-sim test library")
    _test_lib_path = path


def build(jobs: int = 8) -> str:
    """Compile lib/libftar.so, the drivers and ftrun for gfx950 (make, hipcc)."""
    subprocess.run(["make", "-s", "-C", HERE, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    path = _test_lib_path or LIB_PATH
    if not os.path.exists(path):
        raise FtarError(f"{path} is not built: run `make -C {HERE}` (the HIP path has no fallback)")
    L = ctypes.CDLL(path)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    pp = ctypes.POINTER(vp)
    sig = {
        "ftar_init": ([pp], i),
        "ftar_init_rank": ([pp, ctypes.c_char_p, i, i, i], i),
        "ftar_finalize": ([vp], i),
        "ftar_comm_rank": ([vp, ctypes.POINTER(i)], i),
        "ftar_comm_size": ([vp, ctypes.POINTER(i)], i),
        "ftar_world_rank": ([vp, ctypes.POINTER(i)], i),
        "ftar_world_size": ([vp, ctypes.POINTER(i)], i),
        "ftar_comm_device": ([vp, ctypes.POINTER(i)], i),
        "ftar_barrier": ([vp], i),
        "ftar_set_kills": ([vp, ctypes.POINTER(Kill), i], i),
        "ftar_allreduce_rabenseifner": ([vp, vp, sz, i, i, vp], i),
        "ftar_recursive_doubling": ([vp, vp, sz, i, i, vp], i),
        "ftar_allreduce_rabenseifner_host": ([vp, vp, sz, i, i, vp], i),
        "ftar_recursive_doubling_host": ([vp, vp, sz, i, i, vp], i),
        "ftar_reduce_local": ([vp, vp, sz, i, i, vp], i),
        "ftar_set_reduce_variant": ([i], i),
        "ftar_comm_set_stream": ([vp, vp], i),
        "ftar_comm_set_option": ([vp, i, ctypes.c_double], i),
        "ftar_comm_get_option": ([vp, i, ctypes.POINTER(ctypes.c_double)], i),
        "ftar_last_stats": ([vp, ctypes.POINTER(Stats)], i),
        "ftar_set_profiling": ([vp, i], i),
        "ftar_version": ([], ctypes.c_char_p),
    }
    for name, (args, ret) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ret
    L.ftar_abort.argtypes = [vp, i]
    L.ftar_abort.restype = None
    _lib = L
    return L


def _dtype_of(t) -> int:
    import torch
    m = {torch.int32: INT32, torch.float32: FLOAT32, torch.int64: INT64, torch.float64: FLOAT64}
    if t.dtype not in m:
        raise FtarError(f"unsupported dtype {t.dtype}")
    return m[t.dtype]


def _ptr(x):
    """A buffer of the device entry points: a contiguous tensor on the comm's GPU, or a
    pinned host tensor (the kernels read and write it in place over PCIe; include/ftar.h)."""
    if isinstance(x, int):
        return x
    # (host-sim test library: its "device" memory is host memory)
    if not x.is_contiguous() or not (x.is_cuda or _test_lib_path is not None or x.is_pinned()):
        raise FtarError("buffers must be contiguous device tensors or pinned host tensors")
    return x.data_ptr()


def _check(rc: int, what: str):
    if rc != SUCCESS:
        raise FtarError(f"{what} failed with code {rc}")


def reduce_local(inp, inout, count=None, dtype=None, op: int = SUM, stream=None):
    """MPI_Reduce_local(in, inout): inout = inout <op> in on the GPU (asynchronous on
    `stream`, default the current torch stream).  Operands may be pinned host tensors
    (zero copy over PCIe)."""
    if count is None:
        count = inout.numel()
    if dtype is None:
        dtype = _dtype_of(inout)
    if stream is None and not isinstance(inout, int):
        import torch
        dev = inout.device if inout.is_cuda else (inp.device if getattr(inp, "is_cuda", False) else None)
        stream = torch.cuda.current_stream(dev).cuda_stream
    _check(lib().ftar_reduce_local(_ptr(inp), _ptr(inout), count, dtype, op, stream or None),
           "ftar_reduce_local")


def set_reduce_variant(v: int):
    _check(lib().ftar_set_reduce_variant(v), "ftar_set_reduce_variant")


class Comm:
    """An ftar communicator (one per rank process)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def from_env(cls):
        h = ctypes.c_void_p()
        _check(lib().ftar_init(ctypes.byref(h)), "ftar_init")
        return cls(h)

    @classmethod
    def init_rank(cls, job: str, rank: int, size: int, device: int):
        h = ctypes.c_void_p()
        _check(lib().ftar_init_rank(ctypes.byref(h), job.encode(), rank, size, device), "ftar_init_rank")
        return cls(h)

    def _q(self, fn):
        v = ctypes.c_int()
        _check(fn(self._h, ctypes.byref(v)), fn.__name__)
        return v.value

    @property
    def rank(self):
        return self._q(lib().ftar_comm_rank)

    @property
    def size(self):
        return self._q(lib().ftar_comm_size)

    @property
    def world_rank(self):
        return self._q(lib().ftar_world_rank)

    @property
    def world_size(self):
        return self._q(lib().ftar_world_size)

    @property
    def device(self):
        return self._q(lib().ftar_comm_device)

    def barrier(self):
        _check(lib().ftar_barrier(self._h), "ftar_barrier")

    def set_stream(self, stream):
        _check(lib().ftar_comm_set_stream(self._h, stream), "ftar_comm_set_stream")

    def set_option(self, opt: int, value: float):
        """Transport option (collective: same value on every live rank before the next call)."""
        _check(lib().ftar_comm_set_option(self._h, opt, float(value)), "ftar_comm_set_option")

    def get_option(self, opt: int) -> float:
        v = ctypes.c_double()
        _check(lib().ftar_comm_get_option(self._h, opt, ctypes.byref(v)), "ftar_comm_get_option")
        return v.value

    def set_profiling(self, on: bool):
        _check(lib().ftar_set_profiling(self._h, int(on)), "ftar_set_profiling")

    def set_kills(self, kills):
        arr = (Kill * max(1, len(kills)))(*[Kill(*k) for k in kills])
        _check(lib().ftar_set_kills(self._h, arr, len(kills)), "ftar_set_kills")

    def last_stats(self) -> Stats:
        s = Stats()
        _check(lib().ftar_last_stats(self._h, ctypes.byref(s)), "ftar_last_stats")
        return s

    def allreduce_rabenseifner(self, sbuf, rbuf, count=None, dtype=None, op: int = SUM) -> int:
        if count is None:
            count = rbuf.numel()
        if dtype is None:
            dtype = _dtype_of(rbuf)
        return lib().ftar_allreduce_rabenseifner(_ptr(sbuf), _ptr(rbuf), count, dtype, op, self._h)

    def allreduce_rabenseifner_host(self, sbuf, rbuf, count=None, dtype=None, op: int = SUM) -> int:
        """Host buffers (ideally pinned torch CPU tensors): H2D, device Allreduce, D2H."""
        if count is None:
            count = rbuf.numel()
        if dtype is None:
            dtype = _dtype_of(rbuf)
        return lib().ftar_allreduce_rabenseifner_host(sbuf.data_ptr(), rbuf.data_ptr(), count, dtype, op, self._h)

    def recursive_doubling(self, src, dst, count=None, dtype=None, op: int = SUM) -> int:
        if count is None:
            count = dst.numel()
        if dtype is None:
            dtype = _dtype_of(dst)
        return lib().ftar_recursive_doubling(_ptr(src), _ptr(dst), count, dtype, op, self._h)

    def recursive_doubling_host(self, src, dst, count=None, dtype=None, op: int = SUM) -> int:
        """Host buffers (ideally pinned torch CPU tensors)."""
        if count is None:
            count = dst.numel()
        if dtype is None:
            dtype = _dtype_of(dst)
        return lib().ftar_recursive_doubling_host(src.data_ptr(), dst.data_ptr(), count, dtype, op, self._h)

    def finalize(self):
        if self._h:
            _check(lib().ftar_finalize(self._h), "ftar_finalize")
            self._h = None


def version() -> str:
    return lib().ftar_version().decode()
