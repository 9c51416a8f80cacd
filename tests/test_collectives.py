"""CPU tests of the emulated ring collectives beyond all-reduce (ncclReduceScatter, ncclAllGather,
ncclReduce, ncclBroadcast) and of the tree all-reduce (runTreeSplit), include/nexr_ring.h.

As in test_ring.py, every reduceCopy / LL / LL128 step is served by the CPU oracle through the
schedule's function pointers, so the C++ SCHEDULES (chunking, slice/step credits, peer order,
FIFO wrap-around, the tree's two concurrent halves per rank) are checked against oracle/ring.py's
independent restatements, bit for bit, without a GPU.
"""
import ctypes
import importlib

import numpy as np
import pytest

import make_golden as mg

PROTOS = {"simple": 0, "ll": 1, "ll128": 2}
BUFF = {"simple": 64 << 10, "ll": 8 * 1024 * 16, "ll128": 8 * 2048 * 4}  # small: many steps, FIFO wrap


@pytest.fixture(scope="module")
def ring(nexr):
    return importlib.import_module("nex-nccl_amd.ring")


@pytest.fixture(scope="module")
def fns(oracle):
    L = oracle.lib()
    cast = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    return cast(L.oracle_reduce_copy_fn), cast(L.oracle_reduce_copy_ll_fn), cast(L.oracle_reduce_copy_ll128_fn)


def _comm(ring, fns, n, proto, buff=None, ranks_per_node=0, tree_index=0):
    f, fll, fll128 = fns
    return ring.RingComm(n, ring.HOST_MEMORY, BUFF[proto] if buff is None else buff, f, 20000, PROTOS[proto], fll,
                         fll128, ranks_per_node, tree_index)


def _ptrs(arrs):
    return [a.ctypes.data if a is not None else 0 for a in arrs]


def _same(dt, got, exp, what):
    assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp), what


CASES = [(mg.F32, 0, False), (mg.BF16, 0, True), (mg.F16, 4, True), (mg.I32, 3, True), (mg.I8, 1, True),
         (mg.U64, 2, True), (mg.F64, 4, False)]


@pytest.mark.parametrize("proto", ["simple", "ll", "ll128"])
@pytest.mark.parametrize("n_ranks", [2, 3, 5])
@pytest.mark.parametrize("dt,op,special", CASES)
def test_reduce_scatter(ring, oracle, fns, proto, n_ranks, dt, op, special):
    from oracle.ring import reduce_scatter_expected
    recvcount = 9_001 + 5 * n_ranks
    inputs = mg.gen_inputs(dt, n_ranks, recvcount * n_ranks, 0xD00 + 7 * dt + op, special)
    recv = [np.zeros_like(x[:recvcount]) for x in inputs]
    with _comm(ring, fns, n_ranks, proto) as comm:
        comm.reduce_scatter(_ptrs(inputs), _ptrs(recv), recvcount, dt, op)
    exp = reduce_scatter_expected(inputs, dt, op, proto)
    for r in range(n_ranks):
        _same(dt, recv[r], exp[r], f"rank {r}")


@pytest.mark.parametrize("proto", ["simple", "ll", "ll128"])
@pytest.mark.parametrize("n_ranks", [2, 4])
@pytest.mark.parametrize("in_place", [False, True])
def test_all_gather(ring, oracle, fns, proto, n_ranks, in_place):
    from oracle.ring import all_gather_expected
    dt = mg.F16
    count = 12_345
    inputs = mg.gen_inputs(dt, n_ranks, count, 0xE00 + n_ranks, True)  # NaN payloads must survive copies
    recv = [np.zeros(count * n_ranks, dtype=inputs[0].dtype) for _ in range(n_ranks)]
    if in_place:
        for r in range(n_ranks):
            recv[r][r * count:(r + 1) * count] = inputs[r]
        send = [recv[r][r * count:] for r in range(n_ranks)]
    else:
        send = inputs
    with _comm(ring, fns, n_ranks, proto) as comm:
        comm.all_gather(_ptrs(send), _ptrs(recv), count, dt)
    exp = all_gather_expected(inputs)
    for r in range(n_ranks):
        assert recv[r].tobytes() == exp[r].tobytes(), f"rank {r}"


@pytest.mark.parametrize("proto", ["simple", "ll", "ll128"])
@pytest.mark.parametrize("n_ranks,root", [(2, 0), (2, 1), (3, 2), (5, 1)])
@pytest.mark.parametrize("dt,op,special", [(mg.F32, 0, False), (mg.BF16, 4, True), (mg.I32, 2, True)])
def test_reduce(ring, oracle, fns, proto, n_ranks, root, dt, op, special):
    from oracle.ring import reduce_expected
    count = 30_011
    inputs = mg.gen_inputs(dt, n_ranks, count, 0xF00 + 3 * root + dt, special)
    recv = [np.zeros_like(inputs[0]) if r == root else None for r in range(n_ranks)]
    with _comm(ring, fns, n_ranks, proto) as comm:
        comm.reduce(_ptrs(inputs), _ptrs(recv), count, dt, op, root)
    _same(dt, recv[root], reduce_expected(inputs, dt, op, root, proto), "root")


@pytest.mark.parametrize("proto", ["simple", "ll", "ll128"])
@pytest.mark.parametrize("n_ranks,root", [(2, 1), (3, 0), (4, 2)])
@pytest.mark.parametrize("in_place", [False, True])
def test_broadcast(ring, oracle, fns, proto, n_ranks, root, in_place):
    from oracle.ring import broadcast_expected
    dt = mg.BF16
    count = 25_003
    inputs = mg.gen_inputs(dt, n_ranks, count, 0x1000 + root, True)
    recv = [np.zeros_like(inputs[0]) for _ in range(n_ranks)]
    if in_place:
        recv[root] = inputs[root].copy()
    send = [(recv[r] if in_place else inputs[r]) if r == root else None for r in range(n_ranks)]
    with _comm(ring, fns, n_ranks, proto) as comm:
        comm.broadcast(_ptrs(send), _ptrs(recv), count, dt, root)
    exp = broadcast_expected(inputs, root)
    for r in range(n_ranks):
        assert recv[r].tobytes() == exp[r].tobytes(), f"rank {r}"


def test_collectives_one_rank_and_empty(ring, oracle, fns):
    from oracle.ring import reduce_scatter_expected
    x = mg.gen_inputs(mg.F32, 1, 1000, 5, False)
    out = np.zeros_like(x[0])
    with _comm(ring, fns, 1, "simple") as comm:
        comm.reduce_scatter(_ptrs(x), _ptrs([out]), 1000, mg.F32, 4)  # avg of one rank: PreMulSum x 1.0
        _same(mg.F32, out, reduce_scatter_expected(x, mg.F32, 4)[0], "one rank")
        comm.broadcast(_ptrs(x), _ptrs([out]), 0, mg.F32, 0)  # empty: no-op
    with _comm(ring, fns, 3, "simple") as comm:
        z = [np.zeros(0, np.float32)] * 3
        comm.all_gather(_ptrs([np.zeros(1, np.float32)] * 3), _ptrs([np.zeros(3, np.float32)] * 3), 0, mg.F32)
        comm.reduce(_ptrs(z), [0, 0, 0], 0, mg.F32, 0, 1)


def test_collectives_reuse_one_comm(ring, oracle, fns):
    # step counters persist across different collectives on one communicator
    from oracle.ring import reduce_scatter_expected, broadcast_expected, ring_allreduce_expected, reduce_expected
    n, buff = 3, 1 << 14
    with _comm(ring, fns, n, "simple", buff) as comm:
        for it in range(3):
            x = mg.gen_inputs(mg.I32, n, 3 * 5_000, 40 + it, True)
            rs = [np.zeros(5_000, np.uint32) for _ in range(n)]
            comm.reduce_scatter(_ptrs(x), _ptrs(rs), 5_000, mg.I32, 0)
            for r, e in enumerate(reduce_scatter_expected(x, mg.I32, 0)):
                assert np.array_equal(rs[r], e)
            ar = [np.zeros_like(v) for v in x]
            comm.all_reduce(_ptrs(x), _ptrs(ar), x[0].size, mg.I32, 3)
            for r, e in enumerate(ring_allreduce_expected(x, mg.I32, 3, buff)):
                assert np.array_equal(ar[r], e)
            bc = [np.zeros_like(v) for v in x]
            comm.broadcast(_ptrs(x), _ptrs(bc), x[0].size, mg.I32, it % n)
            for r, e in enumerate(broadcast_expected(x, it % n)):
                assert np.array_equal(bc[r], e)
            red = [np.zeros_like(v) for v in x]
            comm.reduce(_ptrs(x), _ptrs(red), x[0].size, mg.I32, 1, (it + 1) % n)
            assert np.array_equal(red[(it + 1) % n], reduce_expected(x, mg.I32, 1, (it + 1) % n))


def test_collectives_reject_bad_arguments(ring, fns, nexr):
    a = np.zeros(64, np.float32)
    with _comm(ring, fns, 3, "simple") as comm:
        with pytest.raises(nexr.NexrError):
            comm.reduce(_ptrs([a] * 3), _ptrs([a] * 3), 16, mg.F32, 0, 3)  # root out of range
        with pytest.raises(nexr.NexrError):
            comm.broadcast([0, a.ctypes.data, 0], _ptrs([a] * 3), 16, mg.F32, 0)  # root has no sendbuff
        with pytest.raises(nexr.NexrError):
            comm.reduce(_ptrs([a] * 3), [a.ctypes.data, 0, a.ctypes.data], 16, mg.F32, 0, 1)  # root has no recvbuff
        with pytest.raises(nexr.NexrError):
            comm.all_gather(_ptrs([a] * 3), _ptrs([a] * 3), 16, 11)  # fp8
    with pytest.raises(nexr.NexrError):
        _comm(ring, fns, 6, "simple", ranks_per_node=4)  # nodes must split the ranks evenly
    with pytest.raises(nexr.NexrError):
        _comm(ring, fns, 4, "simple", tree_index=2)


# ---- tree ------------------------------------------------------------------------------------------

def test_tree_topology_matches_restatement(ring, oracle, fns):
    from oracle.ring import tree_topology
    for n in range(1, 33):
        for L in sorted({0, 1, 2, 4, n}):
            if L and n % L:
                continue
            for t in (0, 1):
                exp = tree_topology(n, L, t)
                with _comm(ring, fns, n, "simple", ranks_per_node=L, tree_index=t) as comm:
                    got = [comm.tree_topology(r) for r in range(n)]
                assert got == exp, (n, L, t)
                # a spanning tree: one root, parent/child links agree, arity <= 3 (2 at the root)
                roots = [r for r in range(n) if exp[r][0] == -1]
                assert len(roots) == 1 and len(exp[roots[0]][1]) <= 2
                for r, (up, down) in enumerate(exp):
                    assert len(down) <= 3
                    if up != -1:
                        assert r in exp[up][1]
                    for d in down:
                        assert exp[d][0] == r


def test_btree_matches_reference_illustration():
    # graph/trees.cc:17-29: the 14-rank btree drawn in the reference's comment
    from oracle.ring import tree_topology
    t = dict(enumerate(tree_topology(14, 1, 0)))
    assert t[0] == (-1, [8])
    assert t[8] == (0, [4, 12])
    assert t[4] == (8, [2, 6]) and t[12] == (8, [10, 13])
    assert t[2] == (4, [1, 3]) and t[6] == (4, [5, 7]) and t[10] == (12, [9, 11])
    assert t[13] == (12, []) and t[1] == (2, [])


TREES = [(2, 0, 0), (5, 0, 0), (3, 1, 0), (8, 1, 0), (8, 1, 1), (13, 1, 0), (13, 1, 1), (8, 2, 0), (12, 4, 1),
         (9, 3, 0)]


@pytest.mark.parametrize("proto", ["simple", "ll", "ll128"])
@pytest.mark.parametrize("n_ranks,per_node,tree_index", TREES)
def test_tree_all_reduce(ring, oracle, fns, proto, n_ranks, per_node, tree_index):
    from oracle.ring import tree_allreduce_expected, tree_topology
    dt, op = [(mg.F32, 0), (mg.BF16, 4), (mg.I32, 3), (mg.F16, 0)][(n_ranks + per_node) % 4]
    count = 20_000 + 17 * n_ranks
    inputs = mg.gen_inputs(dt, n_ranks, count, 0x1100 + n_ranks * 5 + per_node, True)
    recv = [np.zeros_like(x) for x in inputs]
    with _comm(ring, fns, n_ranks, proto, ranks_per_node=per_node, tree_index=tree_index) as comm:
        comm.tree_all_reduce(_ptrs(inputs), _ptrs(recv), count, dt, op)
    exp = tree_allreduce_expected(inputs, dt, op, tree_topology(n_ranks, per_node, tree_index), proto)
    for r in range(n_ranks):
        _same(dt, recv[r], exp[r], f"rank {r}")


def test_tree_all_reduce_arity_three_every_op(ring, oracle, fns):
    # 4 nodes x 2 ranks: node heads reduce their chain child and up to two other heads (K = 4)
    from oracle.ring import tree_allreduce_expected, tree_topology
    links = tree_topology(8, 2, 0)
    assert max(len(d) for _, d in links) == 3
    for dt, op in [(mg.F64, 0), (mg.I8, 1), (mg.U32, 2), (mg.F16, 3), (mg.I64, 4)]:
        inputs = mg.gen_inputs(dt, 8, 7_777, 0x1200 + dt, True)
        recv = [np.zeros_like(x) for x in inputs]
        with _comm(ring, fns, 8, "simple", 1 << 13, ranks_per_node=2) as comm:
            comm.tree_all_reduce(_ptrs(inputs), _ptrs(recv), inputs[0].size, dt, op)
        exp = tree_allreduce_expected(inputs, dt, op, links)
        for r in range(8):
            _same(dt, recv[r], exp[r], f"dt {dt} op {op} rank {r}")


def test_tree_and_ring_share_one_comm(ring, oracle, fns):
    from oracle.ring import tree_allreduce_expected, tree_topology, ring_allreduce_expected
    n, buff = 5, 1 << 14
    with _comm(ring, fns, n, "simple", buff, ranks_per_node=1) as comm:
        for it in range(3):
            x = mg.gen_inputs(mg.F32, n, 11_111, 70 + it, False)
            out = [np.zeros_like(v) for v in x]
            comm.tree_all_reduce(_ptrs(x), _ptrs(out), x[0].size, mg.F32, 0)
            for r, e in enumerate(tree_allreduce_expected(x, mg.F32, 0, tree_topology(n, 1, 0))):
                assert out[r].tobytes() == e.tobytes()
            comm.all_reduce(_ptrs(x), _ptrs(out), x[0].size, mg.F32, 0)
            for r, e in enumerate(ring_allreduce_expected(x, mg.F32, 0, buff)):
                assert out[r].tobytes() == e.tobytes()


@pytest.mark.parametrize("steps", [9, 11, 13, 33, 35])
def test_round_up_returns_credits(ring, oracle, fns, steps):
    """Reduce + Broadcast (1-step slices) leave both ring links at an odd step; the next all-reduce
    (2-step slices, 4-step chunks) rounds every link up, and the receiver must publish the rounded step
    as its head ("return credits in case we rounded up", prims_simple.h:514-517) or the sender waits
    forever for steps nobody sends (9, 13 and 33 steps hung before the fix)."""
    n, count = 2, 1024 * steps  # 1 KiB... 4 KiB steps of uint32: `steps` steps per collective
    x = [np.arange(count * n, dtype=np.uint32) * 7 + k for k in range(n)]
    o = [np.zeros(count * n, np.uint32) for _ in range(n)]
    with _comm(ring, fns, n, "simple", 8 * 4096) as comm:
        comm.reduce(_ptrs(x), _ptrs(o), count, mg.U32, 0, 1)
        comm.broadcast(_ptrs(x), _ptrs(o), count, mg.U32, 1)
        comm.all_reduce(_ptrs(x), _ptrs(o), count, mg.U32, 0)
    for r in range(n):
        assert np.array_equal(o[r][:count], x[0][:count] + x[1][:count])
