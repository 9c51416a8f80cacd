"""GPU tests of the emulated ring collectives (reduce-scatter, all-gather, reduce, broadcast) and the
tree all-reduce with the MI355X kernels underneath: device-memory mode (buffers and FIFOs in HBM,
nexrReduceCopy / nexrReduceCopyLL / nexrReduceCopyLL128 per step) for every protocol, and host-memory
mode (every step through nexrReduceCopyHost). Outputs are compared bit for bit with oracle/ring.py."""
import importlib

import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

BUFF = {0: 1 << 18, 1: 8 * 16 * 512, 2: 8 * 2048 * 8}
PNAME = {0: "simple", 1: "ll", 2: "ll128"}


@pytest.fixture(scope="module")
def ring(nexr):
    assert torch.cuda.is_available()
    return importlib.import_module("nex-nccl_amd.ring")


def _dev(arrs):
    out = [torch.from_numpy(a.copy()).cuda() if a is not None else None for a in arrs]
    torch.cuda.synchronize()
    return out


def _ptrs(ts):
    return [t.data_ptr() if t is not None else 0 for t in ts]


@pytest.mark.parametrize("proto", [0, 1, 2])
@pytest.mark.parametrize("n,dt,op", [(2, mg.F32, 0), (3, mg.BF16, 4), (4, mg.I32, 3), (3, mg.F16, 1)])
def test_reduce_scatter_device(ring, oracle, proto, n, dt, op):
    from oracle.ring import reduce_scatter_expected
    count = 70_001
    inputs = mg.gen_inputs(dt, n, count * n, 0x2000 + dt + op, True)
    send = _dev(inputs)
    recv = [torch.zeros(count, dtype=s.dtype, device=s.device) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, BUFF[proto], protocol=proto) as comm:
        comm.reduce_scatter(_ptrs(send), _ptrs(recv), count, dt, op)
    exp = reduce_scatter_expected(inputs, dt, op, PNAME[proto])
    for r in range(n):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


@pytest.mark.parametrize("proto", [0, 1, 2])
@pytest.mark.parametrize("in_place", [False, True])
def test_all_gather_device(ring, oracle, proto, in_place):
    from oracle.ring import all_gather_expected
    n, dt, count = 3, mg.F16, 50_003
    inputs = mg.gen_inputs(dt, n, count, 0x2100 + proto, True)
    recv = _dev([np.zeros(count * n, dtype=inputs[0].dtype) for _ in range(n)])
    if in_place:
        for r in range(n):
            recv[r][r * count:(r + 1) * count].copy_(torch.from_numpy(inputs[r]))
        send = [recv[r][r * count:] for r in range(n)]
    else:
        send = _dev(inputs)
    torch.cuda.synchronize()
    with ring.RingComm(n, ring.DEVICE_MEMORY, BUFF[proto], protocol=proto) as comm:
        comm.all_gather(_ptrs(send), _ptrs(recv), count, dt)
    exp = all_gather_expected(inputs)
    for r in range(n):
        assert recv[r].cpu().numpy().tobytes() == exp[r].tobytes(), f"rank {r}"


@pytest.mark.parametrize("proto", [0, 1, 2])
@pytest.mark.parametrize("n,root,dt,op", [(3, 0, mg.F32, 0), (4, 2, mg.I8, 2), (2, 1, mg.BF16, 4)])
def test_reduce_and_broadcast_device(ring, oracle, proto, n, root, dt, op):
    from oracle.ring import reduce_expected, broadcast_expected
    count = 90_007
    inputs = mg.gen_inputs(dt, n, count, 0x2200 + root + dt, True)
    send = _dev(inputs)
    red = [torch.zeros_like(send[0]) if r == root else None for r in range(n)]
    bc = [torch.zeros_like(s) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, BUFF[proto], protocol=proto) as comm:
        comm.reduce(_ptrs(send), _ptrs(red), count, dt, op, root)
        comm.broadcast([send[r].data_ptr() if r == root else 0 for r in range(n)], _ptrs(bc), count, dt, root)
    assert mg.canon_bytes(dt, red[root].cpu().numpy()) == mg.canon_bytes(dt, reduce_expected(inputs, dt, op, root,
                                                                                            PNAME[proto]))
    for r, e in enumerate(broadcast_expected(inputs, root)):
        assert bc[r].cpu().numpy().tobytes() == e.tobytes(), f"rank {r}"


@pytest.mark.parametrize("proto", [0, 1, 2])
@pytest.mark.parametrize("n,per_node,tree_index,dt,op", [(2, 0, 0, mg.F32, 0), (5, 1, 0, mg.BF16, 0),
                                                         (8, 2, 0, mg.F32, 0), (6, 1, 1, mg.I32, 3),
                                                         (4, 0, 0, mg.F16, 4)])
def test_tree_all_reduce_device(ring, oracle, proto, n, per_node, tree_index, dt, op):
    from oracle.ring import tree_allreduce_expected, tree_topology
    count = 120_011
    inputs = mg.gen_inputs(dt, n, count, 0x2300 + n + per_node, True)
    send = _dev(inputs)
    recv = [torch.zeros_like(s) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, BUFF[proto], protocol=proto, tree_ranks_per_node=per_node,
                       tree_index=tree_index) as comm:
        comm.tree_all_reduce(_ptrs(send), _ptrs(recv), count, dt, op)
        # a second call on the same communicator, in place on the first result
        comm.tree_all_reduce(_ptrs(recv), _ptrs(recv), count, dt, op)
    links = tree_topology(n, per_node, tree_index)
    exp = tree_allreduce_expected(inputs, dt, op, links, PNAME[proto])
    exp = tree_allreduce_expected(exp, dt, op, links, PNAME[proto])
    for r in range(n):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


def test_host_memory_collectives_through_staging(ring, oracle):
    # the fork's emulated transport: buffers and FIFOs in host memory, every step nexrReduceCopyHost
    from oracle.ring import reduce_scatter_expected, tree_allreduce_expected, tree_topology
    n, dt, op, count = 4, mg.F32, 0, 40_009
    inputs = mg.gen_inputs(dt, n, count * n, 0x2400, False)
    rs = [np.zeros(count, np.float32) for _ in range(n)]
    tr = [np.zeros(count * n, np.float32) for _ in range(n)]
    with ring.RingComm(n, ring.HOST_MEMORY, 1 << 16, tree_ranks_per_node=1) as comm:
        comm.reduce_scatter([a.ctypes.data for a in inputs], [b.ctypes.data for b in rs], count, dt, op)
        comm.tree_all_reduce([a.ctypes.data for a in inputs], [b.ctypes.data for b in tr], count * n, dt, op)
    for r, e in enumerate(reduce_scatter_expected(inputs, dt, op)):
        assert np.array_equal(rs[r].view(np.uint32), e.view(np.uint32)), f"rs rank {r}"
    for r, e in enumerate(tree_allreduce_expected(inputs, dt, op, tree_topology(n, 1, 0))):
        assert np.array_equal(tr[r].view(np.uint32), e.view(np.uint32)), f"tree rank {r}"


def test_mixed_slice_geometries_on_one_device_comm(ring, oracle):
    # Broadcast/Reduce move 1-step slices and can leave a connection at an odd step; the next
    # all-reduce / reduce-scatter (2-step slices) must start at the rounded-up step
    # (prims_simple.h:512-513, :557-558), never with a slice hanging off the FIFO's last slot.
    from oracle.ring import broadcast_expected, ring_allreduce_expected, reduce_scatter_expected, reduce_expected
    n, dt, buff = 3, mg.F32, 1 << 16  # 8 KiB steps
    count = 2 * 2048 + 100            # 3 broadcast chunks: an odd step count is left on some connections
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff) as comm:
        for it in range(3):
            x = mg.gen_inputs(dt, n, count * n, 0x2500 + it, False)
            send = _dev(x)
            bc = [torch.zeros_like(s) for s in send]
            comm.broadcast(_ptrs(send), _ptrs(bc), count + it, dt, it % n)
            ar = [torch.zeros_like(s) for s in send]
            comm.all_reduce(_ptrs(send), _ptrs(ar), count * n, dt, 0)
            rs = [torch.zeros(count, dtype=s.dtype, device=s.device) for s in send]
            comm.reduce_scatter(_ptrs(send), _ptrs(rs), count, dt, 0)
            red = [torch.zeros_like(send[0]) if r == 1 else None for r in range(n)]
            comm.reduce(_ptrs(send), _ptrs(red), count - it, dt, 0, 1)
            for r, e in enumerate(broadcast_expected([v[:count + it] for v in x], it % n)):
                assert bc[r].cpu().numpy()[:count + it].tobytes() == e.tobytes()
            for r, e in enumerate(ring_allreduce_expected(x, dt, 0, buff)):
                assert ar[r].cpu().numpy().tobytes() == e.tobytes()
            for r, e in enumerate(reduce_scatter_expected(x, dt, 0)):
                assert rs[r].cpu().numpy().tobytes() == e.tobytes()
            e = reduce_expected([v[:count - it] for v in x], dt, 0, 1)
            assert red[1].cpu().numpy()[:count - it].tobytes() == e.tobytes()


def test_caller_device_survives_multi_gpu_comm(ring, oracle):
    """Rank r of a device-memory communicator lives on GPU r % nDev, and the entry points select each
    rank's device while they build its stream and FIFO. The caller's current device (PyTorch's too)
    must be the same after create, the collectives and destroy, as NCCL keeps it (init.cc:1873,
    enqueue.cc:2422). Needs two GPUs: skipped on the one-GPU box, runs on a multi-GPU node."""
    n_dev = torch.cuda.device_count()
    if n_dev < 2:
        pytest.skip("needs 2 GPUs")
    n, count = n_dev, 70_001
    inputs = mg.gen_inputs(mg.I32, n, count, 0x5151, False)
    for home in (0, n_dev - 1):
        torch.cuda.set_device(home)
        send = [torch.from_numpy(a.copy()).to(f"cuda:{r}") for r, a in enumerate(inputs)]
        recv = [torch.zeros_like(t) for t in send]
        for t in send:
            torch.cuda.synchronize(t.device)
        with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 18) as comm:
            assert torch.cuda.current_device() == home, "nexrRingCommCreate moved the caller's device"
            comm.all_reduce(_ptrs(send), _ptrs(recv), count, mg.I32, 0)
            assert torch.cuda.current_device() == home, "nexrRingAllReduce moved the caller's device"
            comm.tree_all_reduce(_ptrs(send), _ptrs(recv), count, mg.I32, 0)
            assert torch.cuda.current_device() == home, "nexrTreeAllReduce moved the caller's device"
        assert torch.cuda.current_device() == home, "nexrRingCommDestroy moved the caller's device"
        exp = np.sum(np.stack(inputs).astype(np.int64), axis=0).astype(np.int32)  # wrapping int32 sum, any order
        for r in range(n):
            assert np.array_equal(recv[r].cpu().numpy(), exp), f"rank {r}"
    torch.cuda.set_device(0)
