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
        L.oracle_reduce_copy_emulated.argtypes = [i32, P(vp), i32, P(vp), sz, i32, i32, u64, i32, P(u64), i32, i32, i32]
        L.oracle_reduce_copy_emulated.restype = i32
        L.oracle_reduce_copy_emulated_mt.argtypes = [i32, P(vp), i32, P(vp), sz, i32, i32, u64, i32, P(u64), i32,
                                                     i32, i32, i32]
        L.oracle_reduce_copy_emulated_mt.restype = i32
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
        L.oracle_set_semantics.argtypes = [i32]
        L.oracle_set_semantics.restype = i32
        L.oracle_get_semantics.argtypes = []
        L.oracle_get_semantics.restype = i32
        _lib = L
    return _lib


def _ptrs(arrs):
    a = (ctypes.c_void_p * max(1, len(arrs)))()
    for i, x in enumerate(arrs):
        a[i] = x.ctypes.data
    return a


def reduce_copy(srcs: Sequence[np.ndarray], n_dsts: int, datatype: int, dev_red_op: int, red_op_arg: int = 0,
                pre_op_args: Optional[Sequence[int]] = None, post_op: bool = False, threads: int = 1,
                dsts: Optional[Sequence[np.ndarray]] = None, emulated: Optional[tuple] = None) -> list:
    """Run the oracle on numpy buffers (any dtype view; the bytes are what count). Returns dsts.

    ``emulated=(n_threads, unroll)`` runs the reference's CPU execution of reduceCopy instead of the
    element loop: that many cooperative emulated threads, one after another, over reduceCopyPacks'
    hunk layout (``oracle_reduce_copy_emulated``; ``threads`` > 1 gives each pthread a slice)."""
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
    if emulated is not None:
        nt, unroll = int(emulated[0]), int(emulated[1])
        if threads > 1:
            rc = lib().oracle_reduce_copy_emulated_mt(*args, nt, unroll, int(threads))
        else:
            rc = lib().oracle_reduce_copy_emulated(*args, nt, unroll)
    elif threads > 1:
        rc = lib().oracle_reduce_copy_mt(*args, int(threads))
    else:
        rc = lib().oracle_reduce_copy(*args)
    if rc != 0:
        raise ValueError(f"oracle rejected arguments (rc={rc})")
    return list(dsts)


def set_semantics(mode: int) -> None:
    """Reduction semantics of every later oracle call (0 nccl, 1 fork, 2 shipped: include/nexr.h)."""
    if lib().oracle_set_semantics(int(mode)) != 0:
        raise ValueError(f"bad semantics {mode}")


def get_semantics() -> int:
    return int(lib().oracle_get_semantics())


class semantics:
    """Context manager: run a block under one semantics, restoring the previous one after."""

    def __init__(self, mode: int):
        self.mode = int(mode)

    def __enter__(self):
        self.prev = get_semantics()
        set_semantics(self.mode)
        return self

    def __exit__(self, *exc):
        set_semantics(self.prev)
        return False


def host_to_dev_red_op(op: int, datatype: int, n_ranks: int):
    out = (ctypes.c_uint64 * 2)()
    rc = lib().oracle_host_to_dev_redop(int(op), int(datatype), int(n_ranks), out)
    if rc != 0:
        return None
    return int(out[0]), int(out[1])


def onerank_reference_coverage(n_elts: int, datatype: int) -> int:
    return int(lib().oracle_onerank_reference_coverage(int(n_elts), int(datatype)))


def reduce_copy_ll(src, src_is_input, recv_lines, recv_flags, with_dst, n_send, send_flags, n_elts, datatype,
                   dev_red_op, red_op_arg=0, post_op=False):
    """One LL step on numpy buffers (lines: uint8 arrays of 16 B per line). Returns (rc, dst, sends)."""
    L = lib()
    if not hasattr(L, "_ll_ready"):
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        P = ctypes.POINTER
        L.oracle_reduce_copy_ll.argtypes = [vp, ctypes.c_int, ctypes.c_int, P(vp), P(u32), vp, ctypes.c_int, P(vp),
                                            P(u32), ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                            ctypes.c_int]
        L.oracle_reduce_copy_ll.restype = ctypes.c_int
        L._ll_ready = True
    esz = L.oracle_type_size(int(datatype))
    n_lines = (n_elts * esz + 7) // 8
    dst = np.zeros(n_elts * esz, dtype=np.uint8) if with_dst else None
    sends = [np.zeros(n_lines * 16, dtype=np.uint8) for _ in range(n_send)]
    rl = (ctypes.c_void_p * max(1, len(recv_lines)))(*[x.ctypes.data for x in recv_lines])
    rf = (ctypes.c_uint32 * max(1, len(recv_flags)))(*recv_flags)
    sl = (ctypes.c_void_p * max(1, n_send))(*[x.ctypes.data for x in sends])
    sf = (ctypes.c_uint32 * max(1, len(send_flags)))(*send_flags)
    rc = L.oracle_reduce_copy_ll(src.ctypes.data if src is not None else None, 1 if src_is_input else 0,
                                 len(recv_lines), rl, rf, dst.ctypes.data if dst is not None else None, n_send, sl, sf,
                                 int(n_elts), int(datatype), int(dev_red_op), int(red_op_arg) & 0xFFFFFFFFFFFFFFFF,
                                 1 if post_op else 0)
    return rc, dst, sends


def make_ll_lines(data: np.ndarray, flag: int) -> np.ndarray:
    """Encode raw data bytes as LL lines {data1, flag, data2, flag} (ncclLLFifoLine), zero-padded."""
    raw = np.ascontiguousarray(data).view(np.uint8)
    n_lines = (raw.size + 7) // 8
    padded = np.zeros(n_lines * 8, dtype=np.uint8)
    padded[:raw.size] = raw
    words = padded.view(np.uint32).reshape(n_lines, 2)
    lines = np.empty((n_lines, 4), dtype=np.uint32)
    lines[:, 0] = words[:, 0]
    lines[:, 1] = flag
    lines[:, 2] = words[:, 1]
    lines[:, 3] = flag
    return lines.reshape(-1).view(np.uint8)


LL128_SLICE_BYTES = 2048
LL128_SLICE_DATA = 1920


def reduce_copy_ll128(src, src_is_input, recv_wires, recv_flags, with_dst, n_send, send_flags, n_elts, datatype,
                      dev_red_op, red_op_arg=0, post_op=False):
    """One LL128 step on numpy buffers (wire: uint8 arrays of 2 KiB slices). Returns (rc, dst, sends)."""
    L = lib()
    if not hasattr(L, "_ll128_ready"):
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        P = ctypes.POINTER
        L.oracle_reduce_copy_ll128.argtypes = [vp, ctypes.c_int, ctypes.c_int, P(vp), P(u64), vp, ctypes.c_int,
                                               P(vp), P(u64), ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_uint64, ctypes.c_int]
        L.oracle_reduce_copy_ll128.restype = ctypes.c_int
        L._ll128_ready = True
    esz = L.oracle_type_size(int(datatype))
    n_slices = (n_elts * esz + LL128_SLICE_DATA - 1) // LL128_SLICE_DATA
    dst = np.zeros(n_elts * esz, dtype=np.uint8) if with_dst else None
    sends = [np.zeros(n_slices * LL128_SLICE_BYTES, dtype=np.uint8) for _ in range(n_send)]
    rw = (ctypes.c_void_p * max(1, len(recv_wires)))(*[x.ctypes.data for x in recv_wires])
    rf = (ctypes.c_uint64 * max(1, len(recv_flags)))(*recv_flags)
    sw = (ctypes.c_void_p * max(1, n_send))(*[x.ctypes.data for x in sends])
    sf = (ctypes.c_uint64 * max(1, len(send_flags)))(*send_flags)
    rc = L.oracle_reduce_copy_ll128(src.ctypes.data if src is not None else None, 1 if src_is_input else 0,
                                    len(recv_wires), rw, rf, dst.ctypes.data if dst is not None else None, n_send, sw,
                                    sf, int(n_elts), int(datatype), int(dev_red_op),
                                    int(red_op_arg) & 0xFFFFFFFFFFFFFFFF, 1 if post_op else 0)
    return rc, dst, sends


def make_ll128_wire(data: np.ndarray, flag: int, datatype: int) -> np.ndarray:
    """Encode data into LL128 wire slices via the oracle (a send-only step)."""
    n = data.size
    rc, _, sends = reduce_copy_ll128(np.ascontiguousarray(data), False, [], [], False, 1, [flag], n, datatype, 0)
    assert rc == 0
    return sends[0]
