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


def channel_parts(n_channels: int, count: int, esz: int, traffic_per_byte: int, ll: bool = False):
    """[(channel, offset, count)] of one collective split over `n_channels` channels: the planner's
    cell partition for a task alone in its plan (reference src/enqueue.cc:539-690; trafficPerByte
    of :74-81, x4 for LL) and ncclCollCbdPart's per-channel view (src/include/device.h:946-970)."""
    min_traffic = 16 << 10
    n_max = max(1, n_channels)
    task_traffic = max(min_traffic, count * esz * traffic_per_byte)
    per_channel = max(min_traffic, task_traffic // n_max)
    tpb = traffic_per_byte * (4 if ll else 1)
    cell = _div_up(_div_up(min_traffic, tpb), 16) * 16
    per_cell_elems = cell // esz
    cells = _div_up(count * esz, cell)
    cell_traffic = cell * tpb
    ch0 = 0
    cells_per_ch = min(cells, _div_up(per_channel, cell_traffic))
    lo_cells = cells if ch0 + 1 == n_max else min(cells, _div_up(per_channel, cell_traffic))
    n_mid = (cells - lo_cells) // cells_per_ch
    hi_cells = (cells - lo_cells) % cells_per_ch
    used = (1 if lo_cells else 0) + n_mid + (1 if hi_cells else 0)
    if n_max < ch0 + used:
        n_mid = n_max - ch0 - 2
        cells_per_ch = (cells - lo_cells) // (n_mid + 1)
        hi_cells = cells_per_ch + (cells - lo_cells) % (n_mid + 1)
    if hi_cells == 0 and n_mid != 0:
        hi_cells, n_mid = cells_per_ch, n_mid - 1
    if lo_cells == 0:
        ch0 += 1
        if n_mid == 0:
            lo_cells, hi_cells = hi_cells, 0
        else:
            lo_cells, n_mid = cells_per_ch, n_mid - 1
    mid_count = cells_per_ch * per_cell_elems if n_mid else 0
    lo_count, hi_count = lo_cells * per_cell_elems, hi_cells * per_cell_elems
    excess = cells * per_cell_elems - count
    if hi_count:
        hi_count -= excess
    else:
        lo_count -= excess
    used = (1 if lo_count else 0) + n_mid + (1 if hi_cells else 0)
    parts = []
    for k in range(used):
        if k == 0:
            parts.append((ch0, 0, lo_count))
        elif k == used - 1:
            parts.append((ch0 + k, lo_count + n_mid * mid_count, hi_count))
        else:
            parts.append((ch0 + k, lo_count + (k - 1) * mid_count, mid_count))
    return parts


def ring_allreduce_expected(inputs, datatype: int, op: int, buff_bytes: int = 4 << 20, n_channels: int = 1):
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
    for _, grid, part_count in channel_parts(n_channels, count, esz, 2):
        chunk = step_bytes * 4 // 512 * 512 // esz  # chunkSize aligned to the 512-B grain (enqueue.cc:2062)
        loop = n * chunk
        for elem_off in range(0, part_count, loop):
            rem = part_count - elem_off
            if rem < loop:
                chunk = _align_up(_div_up(rem, n), 16 // esz)
            for c in range(n):
                lo = grid + elem_off + c * chunk
                hi = grid + min(elem_off + c * chunk + chunk, part_count)
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
                               proto: str = "ll", n_channels: int = 1):
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
    for _, grid, part_count in channel_parts(n_channels, count, esz, 2, ll=proto == "ll"):
        _ll_ring_part(step, inputs, out, grid, part_count, esz, buff_bytes, proto, datatype, dev_op, arg)
    return [out.copy() for _ in range(n)]


def _ll_ring_part(step, inputs, out, grid, count, esz, buff_bytes, proto, datatype, dev_op, arg):
    n = len(inputs)
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
            lo = grid + elem_off + c * chunk
            hi = grid + min(elem_off + c * chunk + chunk, count)
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


def tree_allreduce_expected_channels(inputs, datatype: int, op: int, links_of, n_channels: int,
                                     proto: str = "simple"):
    """The tree all-reduce split over channels: each channel folds its part over its own tree,
    `links_of(channel)` (the upper half of 2+ channels runs the other tree of the double binary tree,
    graph/connect.cc:146-160)."""
    n = len(inputs)
    if n == 1 or inputs[0].size == 0:
        return tree_allreduce_expected(inputs, datatype, op, links_of(0), proto)
    out = np.empty_like(inputs[0])
    for ch, grid, cnt in channel_parts(n_channels, inputs[0].size, inputs[0].itemsize, 2, ll=proto == "ll"):
        sl = slice(grid, grid + cnt)
        out[sl] = tree_allreduce_expected([x[sl] for x in inputs], datatype, op, links_of(ch), proto)[0]
    return [out.copy() for _ in range(n)]


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
