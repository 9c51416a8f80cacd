"""TEST INFRASTRUCTURE ONLY — expected results of the reference's ring and tree collectives.

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
    chunk = step_bytes * 4 // 512 * 512 // esz  # chunkSize aligned to the 512-B grain (enqueue.cc:2062)
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
        chunk = (buff_bytes // 8) // 2 // 16 * 16 // esz
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


# ---- the other collectives that reach reduceCopy through genericOp --------------------------------
# Every output element of these schedules goes through the same fold whatever the chunking (each
# chunk of a segment takes the same path through the ranks), so the restatements fold whole
# segments: SIMPLE folds the local (pre-op'd) input FIRST with the received partials
# (prims_simple.h:238-242), LL/LL128 fold the received PEER partial first (prims_ll.h:251-258,
# prims_ll128.h:214-219). Copies (all-gather, broadcast, the down-sweep) move bits unchanged.

def _encode(op, datatype, n):
    enc = host_to_dev_red_op(op, datatype, n)
    if enc is None:
        raise ValueError("op not encodable")
    return enc


def _one_rank(x, datatype, dev_op, arg):
    """ncclLaunchOneRank (onerank.cc:48-83): PreMulSum scales, everything else copies."""
    if dev_op == PREMULSUM:
        return reduce_copy([x], 1, datatype, dev_op, arg, [arg], True)[0]
    return x.copy()


def _fold_node(proto, x, partials, datatype, dev_op, arg, post):
    """One rank's reduce step over its own input `x` and the children's/predecessor's `partials`:
    SIMPLE returns the value array; LL/LL128 return the step's send lines, or the value array when
    `post` (the last step of the chain, which writes the user output)."""
    if proto == "simple":
        return reduce_copy([x] + list(partials), 1, datatype, dev_op, arg, [arg], post)[0]
    from . import reduce_copy_ll, reduce_copy_ll128
    step = reduce_copy_ll if proto == "ll" else reduce_copy_ll128
    rc, dst, sends = step(x, True, list(partials), [1] * len(partials), post, 1, [1], x.size, datatype, dev_op, arg,
                          post)
    assert rc == 0
    return dst.view(x.dtype) if post else sends[0]


def _chain(proto, xs, datatype, dev_op, arg):
    """Fold along a ring chain: xs[0] sends, every following rank reduces, the last one applies the
    post-op and keeps the result."""
    acc = _fold_node(proto, xs[0], [], datatype, dev_op, arg, False)
    for j, x in enumerate(xs[1:]):
        acc = _fold_node(proto, x, [acc], datatype, dev_op, arg, j == len(xs) - 2)
    return acc


def reduce_scatter_expected(inputs, datatype: int, op: int, proto: str = "simple"):
    """runRing of ncclReduceScatter (reduce_scatter.h:12-52): segment d is sent first by rank d+1
    and finished (post-op) at rank d."""
    n = len(inputs)
    dev_op, arg = _encode(op, datatype, n)
    count = inputs[0].size // n
    if n == 1:
        return [_one_rank(inputs[0], datatype, dev_op, arg)]
    outs = []
    for d in range(n):
        seg = slice(d * count, (d + 1) * count)
        if count == 0:
            outs.append(inputs[0][seg].copy())
            continue
        outs.append(_chain(proto, [inputs[(d + k) % n][seg] for k in range(1, n + 1)], datatype, dev_op, arg))
    return outs


def reduce_expected(inputs, datatype: int, op: int, root: int, proto: str = "simple"):
    """runRing of ncclReduce (reduce.h:12-50): the chain starts at root+1 and ends (post-op) at root."""
    n = len(inputs)
    dev_op, arg = _encode(op, datatype, n)
    if n == 1 or inputs[0].size == 0:
        return _one_rank(inputs[0], datatype, dev_op, arg)
    return _chain(proto, [inputs[(root + k) % n] for k in range(1, n + 1)], datatype, dev_op, arg)


def all_gather_expected(inputs):
    """runRing of ncclAllGather (all_gather.h:12-66): every rank gets all inputs in rank order."""
    out = np.concatenate(inputs)
    return [out.copy() for _ in inputs]


def broadcast_expected(inputs, root: int):
    """runRing of ncclBroadcast (broadcast.h:12-58)."""
    return [inputs[root].copy() for _ in inputs]


def tree_topology(n_ranks: int, ranks_per_node: int = 0, tree_index: int = 0):
    """(up, [down...]) of every rank — an independent restatement of the reference's tree:
    ncclGetBtree / ncclGetDtree (graph/trees.cc:31-109) over the node heads, an intra-node chain
    (graph/connect.cc:51-61), children packed by setTreeDown (:111-121)."""
    L = ranks_per_node or n_ranks
    n_nodes = n_ranks // L

    def btree(nr, rank):
        bit = 1
        while bit < nr:
            if bit & rank:
                break
            bit <<= 1
        if rank == 0:
            return -1, -1, (bit >> 1) if nr > 1 else -1
        up = (rank ^ bit) | (bit << 1)
        if up >= nr:
            up = rank ^ bit
        low = bit >> 1
        d0 = -1 if low == 0 else rank - low
        d1 = -1 if low == 0 else rank + low
        while d1 >= nr:
            d1 = -1 if low == 0 else rank + low
            low >>= 1
        return up, d0, d1

    def dtree(nr, rank):
        if tree_index == 0:
            return btree(nr, rank)
        if nr % 2 == 1:
            u, a, b = btree(nr, (rank - 1 + nr) % nr)
            return tuple(-1 if v == -1 else (v + 1) % nr for v in (u, a, b))
        u, a, b = btree(nr, nr - 1 - rank)
        return tuple(-1 if v == -1 else nr - 1 - v for v in (u, a, b))

    links = []
    for r in range(n_ranks):
        node, i = divmod(r, L)
        up = -1 if i == 0 else r - 1
        down = [] if i == L - 1 else [r + 1]
        if i == 0:
            u, d0, d1 = dtree(n_nodes, node)
            if u != -1:
                up = u * L
            down += [d * L for d in (d0, d1) if d != -1]
        links.append((up, down))
    return links


def tree_allreduce_expected(inputs, datatype: int, op: int, links, proto: str = "simple"):
    """runTreeSplit (all_reduce.h:150-230): every rank folds its input with its children's partials
    (in down[] order) and sends up; the root applies the post-op; the result is broadcast down."""
    n = len(inputs)
    dev_op, arg = _encode(op, datatype, n)
    if n == 1:
        return [_one_rank(inputs[0], datatype, dev_op, arg)]
    if inputs[0].size == 0:
        return [inputs[0].copy() for _ in inputs]
    root = next(r for r in range(n) if links[r][0] == -1)

    def up_value(r):
        kids = [up_value(c) for c in links[r][1]]
        return _fold_node(proto, inputs[r], kids, datatype, dev_op, arg, r == root)

    final = up_value(root)
    return [final.copy() for _ in range(n)]
