"""TEST INFRASTRUCTURE ONLY — expected results of the reference's ring all-reduce.

Restates the per-element fold order that runRing (reference src/device/all_reduce.h:12-84)
produces with 1 channel and the ring SIMPLE chunking (chunkCount = stepBytes*4/sizeof(T),
src/enqueue.cc:1993-1996; last loop: alignUp(divUp(rem, nranks), 16/sizeof(T))): chunk c of a loop
starts at rank c+1 (directSend of its pre-op'd input), every following rank folds its own pre-op'd
input FIRST with the received partial (srcs[0] = local, prims_simple.h:240), rank c finishes with
the post-op, and every rank receives the final value. Independent of nex-nccl_amd/csrc/nexr_ring.cpp;
the element arithmetic is the C oracle's.
"""
from __future__ import annotations

import numpy as np

from . import host_to_dev_red_op, reduce_copy

PREMULSUM, SUMPOSTDIV = 3, 4


def _div_up(a: int, b: int) -> int:
    return -(-a // b)


def _align_up(a: int, b: int) -> int:
    return _div_up(a, b) * b


def ring_allreduce_expected(inputs, datatype: int, op: int, buff_bytes: int = 4 << 20):
    n = len(inputs)
    enc = host_to_dev_red_op(op, datatype, n)
    if enc is None:
        raise ValueError("op not encodable")
    dev_op, arg = enc
    count = inputs[0].size
    esz = inputs[0].itemsize
    out = np.empty_like(inputs[0])
    if count == 0:
        return [out.copy() for _ in range(n)]
    if n == 1:
        if dev_op == PREMULSUM:
            out = reduce_copy([inputs[0]], 1, datatype, dev_op, arg, [arg], True)[0]
        else:
            out = inputs[0].copy()
        return [out]
    step_bytes = buff_bytes // 8
    chunk = step_bytes * 4 // esz
    loop = n * chunk
    for elem_off in range(0, count, loop):
        rem = count - elem_off
        if rem < loop:
            chunk = _align_up(_div_up(rem, n), 16 // esz)
        for c in range(n):
            lo = elem_off + c * chunk
            hi = min(elem_off + c * chunk + chunk, count)
            if hi <= lo:
                continue
            sl = slice(lo, hi)
            r = (c + 1) % n
            # directSend: K=1 with the pre-op on the local input
            acc = reduce_copy([inputs[r][sl]], 1, datatype, dev_op, arg, [arg], False)[0]
            for k in range(2, n + 1):
                r = (c + k) % n
                post = k == n  # directRecvReduceCopyDirectSend(postOp=true) at rank c
                acc = reduce_copy([inputs[r][sl], acc], 1, datatype, dev_op, arg, [arg], post)[0]
            out[sl] = acc
    return [out.copy() for _ in range(n)]


def ring_allreduce_expected_ll(inputs, datatype: int, op: int, buff_bytes: int = 8 * 512 * 8 * 16,
                               proto: str = "ll"):
    """The LL / LL128-protocol ring: same runRing schedule (chunk = stepBytes/2 for LL,
    stepBytes/16*15 on the 1920-B grain for LL128, src/enqueue.cc:1997-1999), but every step folds
    with the received PEER partial as the first operand (prims_ll.h:251-258, prims_ll128.h:214-219)."""
    from . import reduce_copy_ll, reduce_copy_ll128
    step = reduce_copy_ll if proto == "ll" else reduce_copy_ll128
    n = len(inputs)
    enc = host_to_dev_red_op(op, datatype, n)
    if enc is None:
        raise ValueError("op not encodable")
    dev_op, arg = enc
    count = inputs[0].size
    esz = inputs[0].itemsize
    if count == 0 or n == 1:
        return ring_allreduce_expected(inputs, datatype, op)
    out = np.empty_like(inputs[0])
    if proto == "ll":
        chunk = (buff_bytes // 8) // 2 // esz
    else:
        chunk = (buff_bytes // 8) // 16 * 15 // 1920 * 1920 // esz
    loop = n * chunk
    for elem_off in range(0, count, loop):
        rem = count - elem_off
        if rem < loop:
            chunk = _align_up(_div_up(rem, n), 16 // esz)
        for c in range(n):
            lo = elem_off + c * chunk
            hi = min(lo + chunk, count)
            if hi <= lo:
                continue
            m = hi - lo
            r = (c + 1) % n
            rc, _, sends = step(inputs[r][lo:hi], True, [], [], False, 1, [1], m, datatype, dev_op, arg)
            for k in range(2, n + 1):
                r = (c + k) % n
                post = k == n
                rc, dst, sends = step(inputs[r][lo:hi], True, [sends[0]], [1], post, 1, [1], m, datatype, dev_op, arg,
                                      post)
                assert rc == 0
            out[lo:hi] = dst.view(out.dtype)
    return [out.copy() for _ in range(n)]
