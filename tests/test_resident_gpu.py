"""GPU tests of the device-resident ring all-reduce (nexrRingAllReduceResident, nexr_resident.hip):
every rank's runRing (src/device/all_reduce.h:12-84) inside one launch, its workgroups waiting on
step counters in HBM. The schedule, chunking and channel split are the host-sequenced ring's, so the
result must equal, bit for bit, both the fold-order oracle (oracle/ring.py) and nexrRingAllReduce on
the same communicator."""
import importlib

import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SUM, PROD, MAX, MIN, AVG = 0, 1, 2, 3, 4


@pytest.fixture(scope="module")
def ring(nexr):
    assert torch.cuda.is_available()
    from conftest import extras_ring
    return extras_ring()  # include/nexr_extras.h: skipped when the opt-in library is not built


def _dev(arrs):
    out = [torch.from_numpy(a.copy()).cuda() for a in arrs]
    torch.cuda.synchronize()
    return out


def _ptrs(ts):
    return [t.data_ptr() for t in ts]


# (ranks, datatype, op, count, buffBytes (0 = 4 MiB), channels)
CASES = [
    (2, mg.F32, SUM, 1 << 20, 0, 1),          # C1's shape
    (3, mg.BF16, SUM, 300_001, 1 << 18, 1),
    (4, mg.I32, MIN, 70_001, 1 << 16, 2),
    (3, mg.F16, AVG, 100_003, 1 << 16, 4),
    (2, mg.I8, MAX, 1_000_003, 0, 2),
    (5, mg.F64, PROD, 40_000, 1 << 16, 1),
    (8, mg.F32, AVG, 65_537, 1 << 16, 3),
    (4, mg.U8, SUM, 17, 1 << 16, 2),
    (2, mg.I64, AVG, 123_457, 1 << 16, 1),
    (6, mg.U32, MAX, 999_999, 1 << 17, 2),
]


@pytest.mark.parametrize("n,dt,op,count,buff,nch", CASES)
def test_resident_matches_oracle_and_host_ring(ring, oracle, n, dt, op, count, buff, nch):
    from oracle.ring import ring_allreduce_expected
    inputs = mg.gen_inputs(dt, n, count, 7 * dt + 13 * op + n, special=True)
    send = _dev(inputs)
    recv = [torch.zeros_like(s) for s in send]
    host = [torch.zeros_like(s) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff, n_channels=nch, timeout_ms=20000) as comm:
        comm.all_reduce_resident(_ptrs(send), _ptrs(recv), count, dt, op)
        comm.all_reduce(_ptrs(send), _ptrs(host), count, dt, op)
    exp = ring_allreduce_expected(inputs, dt, op, buff or (4 << 20), nch)
    for r in range(n):
        got = recv[r].cpu().numpy()
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp[r]), f"rank {r} vs oracle"
        assert np.array_equal(got.view(np.uint8), host[r].cpu().numpy().view(np.uint8)), f"rank {r} vs host ring"


def test_resident_repeated_and_interleaved_with_host_ring(ring, oracle):
    """Step counters persist in HBM across calls (each member resumes from its own records), and the
    host-sequenced ring's FIFOs and counters are independent of them: any interleaving stays exact."""
    from oracle.ring import ring_allreduce_expected
    n, dt, buff = 3, mg.F32, 1 << 16
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff, n_channels=2, timeout_ms=20000) as comm:
        for it, (count, resident) in enumerate([(50_000, True), (7, True), (200_003, False), (131_072, True),
                                                (1, True), (99_999, False), (300_000, True)]):
            inputs = mg.gen_inputs(dt, n, count, 100 + it, special=False)
            send = _dev(inputs)
            recv = [torch.zeros_like(s) for s in send]
            (comm.all_reduce_resident if resident else comm.all_reduce)(_ptrs(send), _ptrs(recv), count, dt, SUM)
            exp = ring_allreduce_expected(inputs, dt, SUM, buff, 2)
            for r in range(n):
                assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), (it, r)


def test_resident_in_place(ring, oracle):
    from oracle.ring import ring_allreduce_expected
    n, dt, count = 4, mg.BF16, 250_001
    inputs = mg.gen_inputs(dt, n, count, 5, special=True)
    buf = _dev(inputs)
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 16, timeout_ms=20000) as comm:
        comm.all_reduce_resident(_ptrs(buf), _ptrs(buf), count, dt, SUM)
    exp = ring_allreduce_expected(inputs, dt, SUM, 1 << 16, 1)
    for r in range(n):
        assert mg.canon_bytes(dt, buf[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), r


def test_resident_misaligned_user_buffers(ring, oracle):
    """User buffers at odd byte offsets: 16-byte user accesses at any alignment (as the SIMPLE kernel),
    FIFO pieces stay aligned."""
    from oracle.ring import ring_allreduce_expected
    n, dt, count = 2, mg.F16, 77_777
    inputs = mg.gen_inputs(dt, n, count, 9, special=True)
    raw_s = [torch.zeros(count * 2 + 64, dtype=torch.uint8, device="cuda") for _ in range(n)]
    raw_r = [torch.zeros(count * 2 + 64, dtype=torch.uint8, device="cuda") for _ in range(n)]
    for r in range(n):
        raw_s[r][3 + r:3 + r + count * 2].copy_(torch.from_numpy(inputs[r].view(np.uint8).copy()).cuda())
    torch.cuda.synchronize()
    sp = [raw_s[r].data_ptr() + 3 + r for r in range(n)]
    rp = [raw_r[r].data_ptr() + 5 + 2 * r for r in range(n)]
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 16, n_channels=2, timeout_ms=20000) as comm:
        comm.all_reduce_resident(sp, rp, count, dt, SUM)
    exp = ring_allreduce_expected(inputs, dt, SUM, 1 << 16, 2)
    for r in range(n):
        got = raw_r[r][5 + 2 * r:5 + 2 * r + count * 2].cpu().numpy().view(np.uint16)
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp[r]), r
        assert int(raw_r[r][:5 + 2 * r].sum()) == 0 and int(raw_r[r][5 + 2 * r + count * 2:].sum()) == 0, "guard bytes"


def test_resident_rejects_what_it_does_not_run(ring):
    with ring.RingComm(2, ring.DEVICE_MEMORY, 0, protocol=ring.PROTO_LL) as comm:
        x = torch.zeros(64, device="cuda")
        with pytest.raises(Exception) as e:
            comm.all_reduce_resident([x.data_ptr()] * 2, [x.data_ptr()] * 2, 64, mg.F32, SUM)
        assert "InvalidUsage" in str(e.value) or "5" in str(e.value)


def test_resident_across_gpus(ring, oracle):
    """Ranks on distinct GPUs (rank r on GPU r mod visible): each GPU runs its ranks' part of the
    schedule in its own launch, FIFO bytes and step counters crossing xGMI. Skipped on one GPU."""
    from oracle.ring import ring_allreduce_expected
    nd = torch.cuda.device_count()
    if nd < 2:
        pytest.skip("needs 2 GPUs")
    n, dt, count = min(nd, 8), mg.F32, 1_000_003
    inputs = mg.gen_inputs(dt, n, count, 77, special=False)
    send = [torch.from_numpy(x.copy()).to(f"cuda:{r}") for r, x in enumerate(inputs)]
    recv = [torch.zeros_like(s) for s in send]
    for r in range(n):
        torch.cuda.synchronize(r)
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 18, n_channels=2, timeout_ms=20000) as comm:
        comm.all_reduce_resident(_ptrs(send), _ptrs(recv), count, dt, SUM)
    exp = ring_allreduce_expected(inputs, dt, SUM, 1 << 18, 2)
    for r in range(n):
        assert recv[r].device.index == r
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), r


def test_resident_uncached_layout_in_a_fresh_process(ring):
    """NEXR_RESIDENT_UNCACHED=1 gives a one-GPU communicator the layout used when ranks span GPUs
    (uncached FIFOs and step records, hipDeviceMallocUncached): the C1 shape and a 4-rank, 2-channel
    bf16 case stay exact. Run in a child process: the switch is read once per process."""
    import os
    import subprocess
    import sys
    code = r'''
import importlib, sys
sys.path.insert(0, "tests/golden")
import numpy as np, torch
import make_golden as mg
from oracle.ring import ring_allreduce_expected
ring = importlib.import_module("nex-nccl_amd.ring")
for n, dt, count, buff, nch in ((2, mg.F32, 1 << 20, 0, 1), (4, mg.BF16, 300_001, 1 << 16, 2)):
    inputs = mg.gen_inputs(dt, n, count, 3 + n, special=True)
    send = [torch.from_numpy(a.copy()).cuda() for a in inputs]
    recv = [torch.zeros_like(s) for s in send]
    torch.cuda.synchronize()
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff, n_channels=nch, timeout_ms=20000, extras=True) as comm:
        for _ in range(3):
            comm.all_reduce_resident([t.data_ptr() for t in send], [t.data_ptr() for t in recv], count, dt, 0)
    exp = ring_allreduce_expected(inputs, dt, 0, buff or (4 << 20), nch)
    assert all(mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]) for r in range(n)), (n, dt)
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NEXR_RESIDENT_UNCACHED="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def _ptrs0(ts):
    return [t.data_ptr() if t is not None else 0 for t in ts]


@pytest.mark.parametrize("n,dt,op,nch", [(2, mg.F32, SUM, 1), (3, mg.BF16, AVG, 2), (4, mg.I32, MIN, 4),
                                         (5, mg.F16, PROD, 1), (8, mg.U8, MAX, 2)])
def test_resident_reduce_scatter(ring, oracle, n, dt, op, nch):
    from oracle.ring import reduce_scatter_expected
    count = 70_001
    inputs = mg.gen_inputs(dt, n, count * n, 0x3000 + dt + op, True)
    send = _dev(inputs)
    recv = [torch.zeros(count, dtype=s.dtype, device=s.device) for s in send]
    host = [torch.zeros_like(r) for r in recv]
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 16, n_channels=nch, timeout_ms=20000) as comm:
        comm.reduce_scatter_resident(_ptrs(send), _ptrs(recv), count, dt, op)
        comm.reduce_scatter(_ptrs(send), _ptrs(host), count, dt, op)
    exp = reduce_scatter_expected(inputs, dt, op, "simple")
    for r in range(n):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"
        assert torch.equal(recv[r].view(torch.uint8), host[r].view(torch.uint8)), f"rank {r} vs host ring"


@pytest.mark.parametrize("n,nch,in_place", [(2, 1, False), (3, 2, True), (4, 4, False), (8, 1, True)])
def test_resident_all_gather(ring, oracle, n, nch, in_place):
    from oracle.ring import all_gather_expected
    dt, count = mg.F16, 50_003
    inputs = mg.gen_inputs(dt, n, count, 0x3100 + n, True)
    recv = _dev([np.zeros(count * n, dtype=inputs[0].dtype) for _ in range(n)])
    if in_place:
        for r in range(n):
            recv[r][r * count:(r + 1) * count].copy_(torch.from_numpy(inputs[r]))
        send = [recv[r][r * count:] for r in range(n)]
    else:
        send = _dev(inputs)
    torch.cuda.synchronize()
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 16, n_channels=nch, timeout_ms=20000) as comm:
        comm.all_gather_resident(_ptrs(send), _ptrs(recv), count, dt)
    exp = all_gather_expected(inputs)
    for r in range(n):
        assert recv[r].cpu().numpy().tobytes() == exp[r].tobytes(), f"rank {r}"


@pytest.mark.parametrize("n,root,dt,op,nch", [(3, 0, mg.F32, SUM, 1), (4, 2, mg.I8, MAX, 2), (2, 1, mg.BF16, AVG, 4),
                                              (6, 5, mg.F64, PROD, 2)])
def test_resident_reduce_and_broadcast(ring, oracle, n, root, dt, op, nch):
    from oracle.ring import reduce_expected, broadcast_expected
    count = 90_007
    inputs = mg.gen_inputs(dt, n, count, 0x3200 + root + dt, True)
    send = _dev(inputs)
    red = [torch.zeros_like(send[0]) if r == root else None for r in range(n)]
    bc = [torch.zeros_like(s) for s in send]
    bc_in_place = [s.clone() if r == root else torch.zeros_like(s) for r, s in enumerate(send)]
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 16, n_channels=nch, timeout_ms=20000) as comm:
        comm.reduce_resident(_ptrs(send), _ptrs0(red), count, dt, op, root)
        comm.broadcast_resident([send[r].data_ptr() if r == root else 0 for r in range(n)], _ptrs(bc), count, dt, root)
        comm.broadcast_resident([bc_in_place[r].data_ptr() if r == root else 0 for r in range(n)], _ptrs(bc_in_place),
                                count, dt, root)
        comm.all_reduce_resident(_ptrs(send), _ptrs(bc_in_place), count, dt, op)  # after Broadcast's 1-step slices
    assert mg.canon_bytes(dt, red[root].cpu().numpy()) == mg.canon_bytes(dt, reduce_expected(inputs, dt, op, root,
                                                                                            "simple"))
    for r, e in enumerate(broadcast_expected(inputs, root)):
        assert bc[r].cpu().numpy().tobytes() == e.tobytes(), f"rank {r}"
    from oracle.ring import ring_allreduce_expected
    exp = ring_allreduce_expected(inputs, dt, op, 1 << 16, nch)
    for r in range(n):
        assert mg.canon_bytes(dt, bc_in_place[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"all-reduce rank {r}"


def test_resident_team_shrinks_to_kernel_occupancy(ring):
    """NEXR_RESIDENT_TEAM=128 with 8 ranks x 2 channels asks for 2,048 workgroups of the int8 kernel
    on one GPU, more than its occupancy lets be resident at once: the team shrinks to fit
    (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs) instead of waiting on workgroups that cannot
    start, and the result stays exact. Child process: the switch is read once per process."""
    import os
    import subprocess
    import sys
    code = r'''
import importlib, sys
sys.path.insert(0, "tests/golden")
import torch
import make_golden as mg
from oracle.ring import ring_allreduce_expected
ring = importlib.import_module("nex-nccl_amd.ring")
n, dt, count, buff, nch = 8, mg.I8, 1_000_003, 1 << 18, 2
inputs = mg.gen_inputs(dt, n, count, 41, special=True)
send = [torch.from_numpy(a.copy()).cuda() for a in inputs]
recv = [torch.zeros_like(s) for s in send]
torch.cuda.synchronize()
with ring.RingComm(n, ring.DEVICE_MEMORY, buff, n_channels=nch, timeout_ms=20000, extras=True) as comm:
    comm.all_reduce_resident([t.data_ptr() for t in send], [t.data_ptr() for t in recv], count, dt, 2)
exp = ring_allreduce_expected(inputs, dt, 2, buff, nch)
assert all(mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]) for r in range(n))
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NEXR_RESIDENT_TEAM="128")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("n,per_node,tree_index,dt,op,nch", [(2, 0, 0, mg.F32, SUM, 1), (5, 1, 0, mg.BF16, SUM, 1),
                                                             (8, 2, 0, mg.F32, SUM, 2), (6, 1, 1, mg.I32, MIN, 1),
                                                             (4, 0, 0, mg.F16, AVG, 4), (7, 1, 0, mg.F64, PROD, 2)])
def test_resident_tree_all_reduce(ring, oracle, n, per_node, tree_index, dt, op, nch):
    """runTreeSplit in one launch: reduce-up and broadcast-down teams per (rank, channel), fan-in up to
    4 (a node head with 3 children), chain and double-binary-tree topologies, both trees (channels in
    the upper half use the other one): equal to nexrTreeAllReduce on the same communicator, bit for
    bit, and to the oracle where one channel makes its expectation channel-free."""
    from oracle.ring import tree_allreduce_expected, tree_topology
    count = 120_011
    inputs = mg.gen_inputs(dt, n, count, 0x3300 + n + per_node, True)
    send = _dev(inputs)
    recv = [torch.zeros_like(s) for s in send]
    host = [torch.zeros_like(s) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, 1 << 16, tree_ranks_per_node=per_node, tree_index=tree_index,
                       n_channels=nch, timeout_ms=20000) as comm:
        comm.tree_all_reduce_resident(_ptrs(send), _ptrs(recv), count, dt, op)
        comm.tree_all_reduce(_ptrs(send), _ptrs(host), count, dt, op)
        again = [torch.zeros_like(s) for s in send]
        comm.tree_all_reduce_resident(_ptrs(send), _ptrs(again), count, dt, op)  # counters resume
    for r in range(n):
        assert torch.equal(recv[r].view(torch.uint8), host[r].view(torch.uint8)), f"rank {r} vs host tree"
        assert torch.equal(again[r].view(torch.uint8), host[r].view(torch.uint8)), f"rank {r}, second call"
    if nch == 1:
        exp = tree_allreduce_expected(inputs, dt, op, tree_topology(n, per_node, tree_index), "simple")
        for r in range(n):
            assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r} vs oracle"
