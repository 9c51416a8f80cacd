"""Multi-channel emulation on MI355X: device-memory communicators with 2-8 channels (each channel
its own FIFOs in HBM, streams and host threads, all running at once), the MI355X reduce-copy under
every step; results bit for bit against the channel-aware restatements."""
import importlib

import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ring(nexr):
    assert torch.cuda.is_available()
    return importlib.import_module("nex-nccl_amd.ring")


def _dev(arrs):
    out = [torch.from_numpy(a.copy()).cuda() for a in arrs]
    torch.cuda.synchronize()
    return out


def _ptrs(ts):
    return [t.data_ptr() for t in ts]


@pytest.mark.parametrize("n,ch,proto", [(2, 2, 0), (3, 4, 0), (4, 8, 0), (3, 2, 1), (4, 4, 2)])
def test_all_reduce_channels_device(ring, oracle, n, ch, proto):
    from oracle.ring import ring_allreduce_expected, ring_allreduce_expected_ll
    rng = np.random.default_rng(n * 10 + ch)
    count = 1 << 20  # C1 size: 4 MiB of fp32 per rank
    inputs = [(rng.standard_normal(count) * 10.0 ** rng.uniform(-4, 4, count)).astype(np.float32) for _ in range(n)]
    send = _dev(inputs)
    recv = [torch.zeros_like(s) for s in send]
    buff = {0: 1 << 20, 1: 8 * 16 * 512, 2: 8 * 2048 * 8}[proto]
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff, protocol=proto, n_channels=ch) as comm:
        comm.all_reduce(_ptrs(send), _ptrs(recv), count, mg.F32, 0)
    if proto == 0:
        exp = ring_allreduce_expected(inputs, mg.F32, 0, buff, n_channels=ch)
    else:
        exp = ring_allreduce_expected_ll(inputs, mg.F32, 0, buff, "ll" if proto == 1 else "ll128", n_channels=ch)
    for r in range(n):
        assert recv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize("n,per_node,ch", [(4, 1, 2), (6, 2, 4)])
def test_tree_channels_device(ring, oracle, n, per_node, ch):
    from oracle.ring import tree_allreduce_expected_channels, tree_topology
    count = 300_007
    inputs = mg.gen_inputs(mg.BF16, n, count, 0x8100 + n, True)
    send = _dev(inputs)
    recv = [torch.zeros_like(s) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 18, tree_ranks_per_node=per_node, n_channels=ch) as comm:
        comm.tree_all_reduce(_ptrs(send), _ptrs(recv), count, mg.BF16, 0)
    exp = tree_allreduce_expected_channels(
        inputs, mg.BF16, 0, lambda k: tree_topology(n, per_node, 1 if (ch >= 2 and k >= ch // 2) else 0), ch)
    for r in range(n):
        assert mg.canon_bytes(mg.BF16, recv[r].cpu().numpy()) == mg.canon_bytes(mg.BF16, exp[r]), r


@pytest.mark.parametrize("n,ch", [(4, 2), (8, 4)])
def test_ring_reduce_scatter_channels_device(ring, oracle, n, ch):
    from oracle.ring import reduce_scatter_expected
    rc, buff = 100_003, 1 << 18
    inputs = mg.gen_inputs(mg.F32, n, rc * n, 0x8200 + n, True)
    send = _dev(inputs)
    recv = [torch.zeros(rc, dtype=s.dtype, device=s.device) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff, n_channels=ch) as comm:
        comm.reduce_scatter(_ptrs(send), _ptrs(recv), rc, mg.F32, 0)
        for r, e in enumerate(reduce_scatter_expected(inputs, mg.F32, 0)):
            assert mg.canon_bytes(mg.F32, recv[r].cpu().numpy()) == mg.canon_bytes(mg.F32, e), r
