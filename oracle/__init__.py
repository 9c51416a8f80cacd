"""TEST INFRASTRUCTURE ONLY — the CPU oracle (checker) for the reduce-copy hot path.

Loads ``oracle/liboracle.so`` (built from ``nexr_oracle.c`` by ``make -C oracle``), a plain-C
restatement of the reference's reduceCopy element loop and scalar arithmetic (citations in the C
file's header). Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / CPU baseline — never as the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, i32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
        P = ctypes.POINTER
        L.oracle_reduce_copy.argtypes = [i32, P(vp), i32, P(vp), sz, i32, i32, u64, i32, P(u64), i32]
        L.oracle_reduce_copy.restype = i32
        L.oracle_reduce_copy_mt.argtypes = [i32, P(vp), i32, P(vp), sz, i32, i32, u64, i32, P(u64), i32, i32]
        L.oracle_reduce_copy_mt.restype = i32
        L.oracle_host_to_dev_redop.argtypes = [i32, i32, i32, P(u64)]
        L.oracle_host_to_dev_redop.restype = i32
        L.oracle_onerank_reference_coverage.argtypes = [sz, i32]
        L.oracle_onerank_reference_coverage.restype = sz
        L.oracle_half_to_float.argtypes = [ctypes.c_uint16]
        L.oracle_half_to_float.restype = ctypes.c_float
        L.oracle_float_to_half.argtypes = [ctypes.c_float]
        L.oracle_float_to_half.restype = ctypes.c_uint16
        L.oracle_float_to_bf16.argtypes = [ctypes.c_float]
        L.oracle_float_to_bf16.restype = ctypes.c_uint16
        L.oracle_type_size.argtypes = [i32]
        L.oracle_type_size.restype = sz
        _lib = L
    return _lib


def _ptrs(arrs):
    a = (ctypes.c_void_p * max(1, len(arrs)))()
    for i, x in enumerate(arrs):
        a[i] = x.ctypes.data
    return a


def reduce_copy(srcs: Sequence[np.ndarray], n_dsts: int, datatype: int, dev_red_op: int, red_op_arg: int = 0,
                pre_op_args: Optional[Sequence[int]] = None, post_op: bool = False, threads: int = 1,
                dsts: Optional[Sequence[np.ndarray]] = None) -> list:
    """Run the oracle on numpy buffers (any dtype view; the bytes are what count). Returns dsts."""
    srcs = [np.ascontiguousarray(s) for s in srcs]
    n_bytes = srcs[0].nbytes
    esz = lib().oracle_type_size(int(datatype))
    if esz == 0:
        raise ValueError("bad datatype")
    n = n_bytes // esz
    if dsts is None:
        dsts = [np.empty_like(srcs[0]) for _ in range(n_dsts)]
    pre = list(pre_op_args or [])
    pre_arr = (ctypes.c_uint64 * len(pre))(*[int(v) & 0xFFFFFFFFFFFFFFFF for v in pre]) if pre else None
    args = [len(srcs), _ptrs(srcs), len(dsts), _ptrs(dsts), n, int(datatype), int(dev_red_op),
            int(red_op_arg) & 0xFFFFFFFFFFFFFFFF, len(pre), pre_arr, 1 if post_op else 0]
    if threads > 1:
        rc = lib().oracle_reduce_copy_mt(*args, int(threads))
    else:
        rc = lib().oracle_reduce_copy(*args)
    if rc != 0:
        raise ValueError(f"oracle rejected arguments (rc={rc})")
    return list(dsts)


def host_to_dev_red_op(op: int, datatype: int, n_ranks: int):
    out = (ctypes.c_uint64 * 2)()
    rc = lib().oracle_host_to_dev_redop(int(op), int(datatype), int(n_ranks), out)
    if rc != 0:
        return None
    return int(out[0]), int(out[1])


def onerank_reference_coverage(n_elts: int, datatype: int) -> int:
    return int(lib().oracle_onerank_reference_coverage(int(n_elts), int(datatype)))
