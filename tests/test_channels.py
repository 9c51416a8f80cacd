"""Multi-channel emulation (nexrRingConfig.nChannels): every collective split over channels the way
the reference's planner splits it (scheduleCollTasksToPlan's cell partition, src/enqueue.cc:539-690,
read back through ncclCollCbdPart, device.h:946-970), each channel with its own links, FIFOs, host
threads and tree (the upper half of the channels on the other tree of the double binary tree,
graph/connect.cc:146-160). CPU tests: the oracle serves every step; float results are compared bit
for bit with the channel-aware restatements in oracle/ring.py."""
import ctypes
import importlib

import numpy as np
import pytest

import make_golden as mg


@pytest.fixture(scope="module")
def ring(nexr):
    return importlib.import_module("nex-nccl_amd.ring")


@pytest.fixture(scope="module")
def fns(oracle):
    L = oracle.lib()
    cast = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    return cast(L.oracle_reduce_copy_fn), cast(L.oracle_reduce_copy_ll_fn), cast(L.oracle_reduce_copy_ll128_fn)


def _ptrs(arrs):
    return [a.ctypes.data if a is not None else 0 for a in arrs]


def _comm(ring, fns, n, ch, proto=0, buff=None, per_node=0, tree_index=0):
    f, fll, fll128 = fns
    buff = buff or {0: 64 << 10, 1: 8 * 1024 * 16, 2: 8 * 2048 * 4}[proto]
    return ring.RingComm(n, ring.HOST_MEMORY, buff, f, 20000, proto, fll, fll128, per_node, tree_index, ch)


def test_channel_parts_cover_the_data():
    from oracle.ring import channel_parts
    for nch in (1, 2, 3, 4, 8, 16, 32, 64):
        for count in (1, 7, 1000, 4096, 65_537, 1 << 20, 3_000_017):
            for esz in (1, 2, 4, 8):
                for tpb, ll in ((1, False), (2, False), (2, True), (4, False), (8, False)):
                    parts = channel_parts(nch, count, esz, tpb, ll)
                    assert 1 <= len(parts) <= nch
                    assert [p[0] for p in parts] == list(range(len(parts)))
                    off = 0
                    for _, o, c in parts:
                        assert o == off and c > 0
                        off += c
                    assert off == count
    # small collectives stay on one channel (16 KiB of traffic at least per channel, :539)
    assert len(channel_parts(8, 1024, 4, 2)) == 1
    assert len(channel_parts(8, 1 << 20, 4, 2)) == 8


@pytest.mark.parametrize("n,ch", [(2, 2), (3, 4), (4, 8), (5, 3)])
@pytest.mark.parametrize("dt,op,special", [(mg.F32, 0, False), (mg.BF16, 0, True), (mg.I32, 2, True)])
def test_ring_all_reduce_channels(ring, oracle, fns, n, ch, dt, op, special):
    from oracle.ring import ring_allreduce_expected
    count = 70_001
    inputs = mg.gen_inputs(dt, n, count, 0x7700 + n * ch + dt, special)
    out = [np.zeros_like(x) for x in inputs]
    with _comm(ring, fns, n, ch) as comm:
        comm.all_reduce(_ptrs(inputs), _ptrs(out), count, dt, op)
    exp = ring_allreduce_expected(inputs, dt, op, 64 << 10, n_channels=ch)
    for r in range(n):
        assert mg.canon_bytes(dt, out[r]) == mg.canon_bytes(dt, exp[r]), r


@pytest.mark.parametrize("n,ch", [(3, 4), (4, 2), (6, 8)])
def test_channel_split_decides_the_fold_order(ring, oracle, fns, n, ch):
    """Wide-range floats make the fold order visible: the emulation equals the restatement with the
    reference's channel split and differs from the single-channel order."""
    from oracle.ring import ring_allreduce_expected
    rng = np.random.default_rng(n * 100 + ch)
    count = 80_000
    inputs = [(rng.standard_normal(count) * 10.0 ** rng.uniform(-4, 4, count)).astype(np.float32) for _ in range(n)]
    out = [np.zeros_like(x) for x in inputs]
    with _comm(ring, fns, n, ch) as comm:
        comm.all_reduce(_ptrs(inputs), _ptrs(out), count, mg.F32, 0)
    exp = ring_allreduce_expected(inputs, mg.F32, 0, 64 << 10, n_channels=ch)
    one = ring_allreduce_expected(inputs, mg.F32, 0, 64 << 10, n_channels=1)
    for r in range(n):
        assert out[r].tobytes() == exp[r].tobytes(), r
    assert any(out[r].tobytes() != one[r].tobytes() for r in range(n))


@pytest.mark.parametrize("proto", [1, 2])
def test_ll_ring_all_reduce_channels(ring, oracle, fns, proto):
    from oracle.ring import ring_allreduce_expected_ll
    n, ch, dt, count = 3, 4, mg.F32, 90_001
    inputs = mg.gen_inputs(dt, n, count, 0x7800 + proto, False)
    out = [np.zeros_like(x) for x in inputs]
    buff = {1: 8 * 1024 * 16, 2: 8 * 2048 * 4}[proto]
    with _comm(ring, fns, n, ch, proto) as comm:
        comm.all_reduce(_ptrs(inputs), _ptrs(out), count, dt, 0)
    exp = ring_allreduce_expected_ll(inputs, dt, 0, buff, "ll" if proto == 1 else "ll128", n_channels=ch)
    for r in range(n):
        assert out[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize("n,per_node,ch", [(4, 1, 2), (6, 2, 4), (8, 1, 4), (5, 0, 2)])
def test_tree_all_reduce_channels(ring, oracle, fns, n, per_node, ch):
    from oracle.ring import tree_allreduce_expected_channels, tree_topology
    dt, count = mg.F32, 60_013
    inputs = mg.gen_inputs(dt, n, count, 0x7900 + n, False)
    out = [np.zeros_like(x) for x in inputs]
    with _comm(ring, fns, n, ch, per_node=per_node) as comm:
        comm.tree_all_reduce(_ptrs(inputs), _ptrs(out), count, dt, 0)

    def links_of(k):
        return tree_topology(n, per_node, 1 if (ch >= 2 and k >= ch // 2) else 0)

    exp = tree_allreduce_expected_channels(inputs, dt, 0, links_of, ch)
    for r in range(n):
        assert out[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize("proto", [0, 1, 2])
def test_other_ring_collectives_channels(ring, oracle, fns, proto):
    from oracle.ring import reduce_scatter_expected, reduce_expected, all_gather_expected, broadcast_expected
    pname = {0: "simple", 1: "ll", 2: "ll128"}[proto]
    n, ch, dt = 4, 3, mg.BF16
    rc = 20_011
    inputs = mg.gen_inputs(dt, n, rc * n, 0x7A00 + proto, True)
    with _comm(ring, fns, n, ch, proto) as comm:
        out = [np.zeros_like(x[:rc]) for x in inputs]
        comm.reduce_scatter(_ptrs(inputs), _ptrs(out), rc, dt, 0)
        for r, e in enumerate(reduce_scatter_expected(inputs, dt, 0, pname)):
            assert mg.canon_bytes(dt, out[r]) == mg.canon_bytes(dt, e)
        ag = [np.zeros(rc * n, dtype=inputs[0].dtype) for _ in range(n)]
        comm.all_gather(_ptrs([x[:rc] for x in inputs]), _ptrs(ag), rc, dt)
        for r, e in enumerate(all_gather_expected([x[:rc] for x in inputs])):
            assert ag[r].tobytes() == e.tobytes()
        red = [np.zeros_like(inputs[0]) for _ in range(n)]
        comm.reduce(_ptrs(inputs), _ptrs(red), rc * n, dt, 1, 2)
        assert mg.canon_bytes(dt, red[2]) == mg.canon_bytes(dt, reduce_expected(inputs, dt, 1, 2, pname))
        bc = [np.zeros_like(inputs[0]) for _ in range(n)]
        comm.broadcast(_ptrs(inputs), _ptrs(bc), rc * n, dt, 1)
        for r, e in enumerate(broadcast_expected(inputs, 1)):
            assert bc[r].tobytes() == e.tobytes()


def test_channels_mixed_collectives_and_reuse(ring, oracle, fns):
    """Several channels on one communicator across collectives (counters carried per channel); integer
    sums are exact whatever the order."""
    n, ch = 4, 4
    rng = np.random.default_rng(5)
    with _comm(ring, fns, n, ch) as comm:
        for it in range(4):
            count = int(rng.integers(1, 200_000))
            x = [rng.integers(0, 1 << 32, count * n, dtype=np.uint64).astype(np.uint32) for _ in range(n)]
            total = (sum(v.astype(np.uint64) for v in x) & 0xFFFFFFFF).astype(np.uint32)
            o = [np.zeros(count * n, np.uint32) for _ in range(n)]
            comm.all_reduce(_ptrs(x), _ptrs(o), count, 3, 0)
            assert all(np.array_equal(v[:count], total[:count]) for v in o)
            comm.tree_all_reduce(_ptrs(x), _ptrs(o), count, 3, 0)
            assert all(np.array_equal(v[:count], total[:count]) for v in o)
            comm.all_gather(_ptrs([v[:count] for v in x]), _ptrs(o), count, 3)
            assert all(np.array_equal(o[r], np.concatenate([v[:count] for v in x])) for r in range(n))
            comm.reduce_scatter(_ptrs(x), _ptrs(o), count, 3, 0)
            assert all(np.array_equal(o[r][:count], total[r * count:(r + 1) * count]) for r in range(n))


def test_channel_limits(ring, fns, nexr):
    with pytest.raises(nexr.NexrError):
        _comm(ring, fns, 2, 65)
    with pytest.raises(nexr.NexrError):
        _comm(ring, fns, 2, -1)
    with _comm(ring, fns, 2, 64) as comm:  # MAXCHANNELS
        x = [np.arange(1 << 20, dtype=np.uint32) + r for r in range(2)]
        o = [np.zeros_like(v) for v in x]
        comm.all_reduce(_ptrs(x), _ptrs(o), 1 << 20, 3, 0)
        assert all(np.array_equal(v, x[0] + x[1]) for v in o)
