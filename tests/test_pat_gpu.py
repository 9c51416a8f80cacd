"""GPU tests of the PAT ReduceScatter / AllGather (nexrPatReduceScatter / nexrPatAllGather) with the
MI355X reduce-copy kernel underneath: buffers and FIFOs in HBM (every step a nexrReduceCopy launch
on the rank's stream, one synchronisation per lock-step batch) and in host memory (every step through
nexrReduceCopyHost). Outputs are compared bit for bit with oracle/pat.py's restatement."""
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


@pytest.mark.parametrize("n,dt,op,count,buff", [
    (2, mg.F32, 0, 100_003, 1 << 18),
    (3, mg.BF16, 0, 40_001, 1 << 16),
    (4, mg.F16, 1, 25_000, 1 << 15),
    (5, mg.I32, 2, 30_011, 1 << 16),
    (8, mg.I8, 3, 50_000, 1 << 15),
    (8, mg.F32, 0, 1 << 20, 0),        # default 4 MiB buffer: 512 KiB steps
    (16, mg.F32, 0, 40, 4 << 20),      # aggregated: 8 worker groups per batch
    (32, mg.BF16, 2, 1000, 4096),      # stepOffset up to 3
])
def test_pat_reduce_scatter_device(ring, oracle, n, dt, op, count, buff):
    from oracle import pat
    inputs = mg.gen_inputs(dt, n, count * n, 0x4100 + n + dt + op, True)
    send = _dev(inputs)
    recv = [torch.zeros(count, dtype=s.dtype, device=s.device) for s in send]
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff) as comm:
        comm.pat_reduce_scatter(_ptrs(send), _ptrs(recv), count, dt, op)
    dev_op, arg = oracle.host_to_dev_red_op(op, dt, n)
    exp = pat.reduce_scatter_expected(inputs, dt, dev_op, arg, (buff or (4 << 20)) // 8)
    for r in range(n):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


@pytest.mark.parametrize("n,count,buff", [(2, 70_001, 1 << 16), (4, 33_333, 1 << 15), (8, 1 << 18, 0),
                                          (16, 40, 4 << 20), (32, 1000, 4096)])
@pytest.mark.parametrize("in_place", [False, True])
def test_pat_all_gather_device(ring, n, count, buff, in_place):
    dt = mg.F16
    inputs = mg.gen_inputs(dt, n, count, 0x4200 + n, True)  # NaN payloads must survive copies
    recv = _dev([np.zeros(count * n, dtype=inputs[0].dtype) for _ in range(n)])
    if in_place:
        for r in range(n):
            recv[r][r * count:(r + 1) * count].copy_(torch.from_numpy(inputs[r]))
        send = [recv[r][r * count:] for r in range(n)]
    else:
        send = _dev(inputs)
    torch.cuda.synchronize()
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff) as comm:
        comm.pat_all_gather(_ptrs(send), _ptrs(recv), count, dt)
    exp = np.concatenate(inputs).tobytes()
    for r in range(n):
        assert recv[r].cpu().numpy().tobytes() == exp, f"rank {r}"


def test_pat_host_memory_through_staging(ring, oracle):
    from oracle import pat
    n, count, buff, dt = 4, 20_000, 1 << 16, mg.F32
    inputs = mg.gen_inputs(dt, n, count * n, 0x4300, False)
    recv = [np.zeros(count, np.float32) for _ in range(n)]
    with ring.RingComm(n, ring.HOST_MEMORY, buff) as comm:
        comm.pat_reduce_scatter([x.ctypes.data for x in inputs], [x.ctypes.data for x in recv], count, dt, 0)
        ag = [np.zeros(count * n, np.float32) for _ in range(n)]
        comm.pat_all_gather([x.ctypes.data for x in recv], [x.ctypes.data for x in ag], count, dt)
    exp = pat.reduce_scatter_expected(inputs, dt, 0, 0, buff // 8)
    for r in range(n):
        assert recv[r].tobytes() == exp[r].tobytes()
        assert ag[r].tobytes() == np.concatenate(exp).tobytes()


def test_pat_and_ring_on_one_device_comm(ring, oracle):
    """PAT's r -> r+1 link is the ring's connection: ring and PAT calls interleave on one comm."""
    from oracle import pat
    from oracle.ring import reduce_scatter_expected
    n, count, buff, dt = 4, 12_345, 1 << 15, mg.BF16
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff) as comm:
        for it in range(2):
            inputs = mg.gen_inputs(dt, n, count * n, 0x4400 + it, True)
            send = _dev(inputs)
            recv = [torch.zeros(count, dtype=s.dtype, device=s.device) for s in send]
            comm.pat_reduce_scatter(_ptrs(send), _ptrs(recv), count, dt, 0)
            for r, e in enumerate(pat.reduce_scatter_expected(inputs, dt, 0, 0, buff // 8)):
                assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, e)
            comm.reduce_scatter(_ptrs(send), _ptrs(recv), count, dt, 0)
            for r, e in enumerate(reduce_scatter_expected(inputs, dt, 0)):
                assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, e)
