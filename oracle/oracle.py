"""ctypes front-end of the CPU oracle (oracle/ftar_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline.  The product path
(fault-tolerant_amd/, libftar.so) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libftar_oracle.so")

INT32, FLOAT32, INT64, FLOAT64 = 0, 1, 2, 3
SUM, PROD, MAX, MIN = 0, 1, 2, 3
LAND, BAND, LOR, BOR, LXOR, BXOR = 4, 5, 6, 7, 8, 9  # MPI logical / bitwise ops (integer types)
PH_PRE, PH_LOOP, PH_AG, PH_POST = 0, 1, 2, 3
PT_BEFORE, PT_AFTER, PT_BARRIER, PT_DURING = 0, 1, 2, 3
OK, DEAD, ABORTED = 0, 1, 2
MAX_RANKS = 64

NP_DTYPE = {INT32: np.int32, FLOAT32: np.float32, INT64: np.int64, FLOAT64: np.float64}
DTYPE_OF = {np.dtype(v): k for k, v in NP_DTYPE.items()}


class Kill(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int), ("phase", ctypes.c_int),
                ("step", ctypes.c_int), ("point", ctypes.c_int)]


class _Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int * MAX_RANKS), ("aborted", ctypes.c_int),
                ("abort_code", ctypes.c_int), ("recoveries", ctypes.c_int),
                ("deviations", ctypes.c_int), ("ret", ctypes.c_int),
                ("size_after", ctypes.c_int), ("order_after", ctypes.c_int * MAX_RANKS)]


@dataclass
class Result:
    status: list
    aborted: bool
    abort_code: int
    recoveries: int
    deviations: int
    ret: int
    order_after: list
    outputs: list = field(default_factory=list)


_lib = None


def build() -> str:
    """Compile the oracle with the committed recipe (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        _lib.ftar_oracle_reduce_local.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_size_t]
        _lib.ftar_oracle_checksum17.argtypes = [vp, ctypes.c_size_t]
        _lib.ftar_oracle_checksum17.restype = ctypes.c_int32
        _lib.ftar_oracle_checksum17_f32.argtypes = [vp, ctypes.c_size_t]
        _lib.ftar_oracle_checksum17_f32.restype = ctypes.c_int32
        for fn in (_lib.ftar_oracle_rabenseifner, _lib.ftar_oracle_recursive_doubling):
            fn.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                           ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(Kill),
                           ctypes.c_int, ctypes.POINTER(_Result)]
    return _lib


def reduce_local(inp: np.ndarray, inout: np.ndarray, op: int = SUM) -> None:
    """MPI_Reduce_local semantics: inout = inout <op> in (in place)."""
    assert inp.dtype == inout.dtype and inp.size == inout.size
    assert inp.flags.c_contiguous and inout.flags.c_contiguous
    lib().ftar_oracle_reduce_local(DTYPE_OF[inp.dtype], op, inp.ctypes.data, inout.ctypes.data, inp.size)


def checksum17(result: np.ndarray) -> int:
    """int res = sum_i result[i] % 17 of the reference drivers."""
    result = np.ascontiguousarray(result)
    if result.dtype == np.float32:
        return int(lib().ftar_oracle_checksum17_f32(result.ctypes.data, result.size))
    assert result.dtype == np.int32
    return int(lib().ftar_oracle_checksum17(result.ctypes.data, result.size))


def expected_checksum(n_ranks: int, count: int) -> int:
    """Closed form of analysis/check_fault.py:62-67 (calcExpectedRes(N-1, BUF_SIZE)),
    wrapped to the driver's 32-bit int as recorded in data/data_compare/*.csv."""
    v = ((n_ranks * (n_ranks - 1) // 2) % 17) * count
    return (v + 2**31) % 2**32 - 2**31


def _run(fn, inputs, kills, op):
    p = len(inputs)
    count = inputs[0].size
    dt = DTYPE_OF[inputs[0].dtype]
    ins = [np.ascontiguousarray(x) for x in inputs]
    outs = [np.zeros_like(x) for x in ins]
    vp = ctypes.c_void_p
    in_arr = (vp * p)(*[x.ctypes.data for x in ins])
    out_arr = (vp * p)(*[x.ctypes.data for x in outs])
    ks = list(kills or [])
    k_arr = (Kill * max(1, len(ks)))(*[Kill(*k) for k in ks])
    res = _Result()
    fn(p, count, dt, op, in_arr, out_arr, k_arr, len(ks), ctypes.byref(res))
    return Result(status=list(res.status[:p]), aborted=bool(res.aborted), abort_code=res.abort_code,
                  recoveries=res.recoveries, deviations=res.deviations, ret=res.ret,
                  order_after=list(res.order_after[:res.size_after]), outputs=outs)


def rabenseifner(inputs, kills=(), op: int = SUM) -> Result:
    """Fault-tolerant Rabenseifner (src/raben) on a list of per-rank numpy vectors.
    kills: iterable of (rank, phase, step, point)."""
    return _run(lib().ftar_oracle_rabenseifner, inputs, kills, op)


def recursive_doubling(inputs, kills=(), op: int = SUM) -> Result:
    """Fault-tolerant recursive doubling (src/rd) on a list of per-rank numpy vectors."""
    return _run(lib().ftar_oracle_recursive_doubling, inputs, kills, op)


def rank_inputs(p: int, count: int, dtype=np.int32):
    """The reference drivers' inputs: buffer[i] = rank (rd/recursive_doubling.c:112-115)."""
    return [np.full(count, r, dtype=dtype) for r in range(p)]


def random_inputs(p: int, count: int, seed: int = 42, dtype=np.float32):
    """Uniform [-1, 1) vectors per rank (SURVEY.md 8d synthetic inputs)."""
    rng = np.random.default_rng(seed)
    if np.dtype(dtype).kind == "f":
        return [(rng.random(count, dtype=np.float64) * 2 - 1).astype(dtype) for _ in range(p)]
    return [rng.integers(-2**20, 2**20, size=count).astype(dtype) for _ in range(p)]
