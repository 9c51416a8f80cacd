"""Runs of LL steps with the credits on the device (nexrReduceCopyLLSteps, ABI 0.3; reference
src/device/prims_ll.h:55-83 waitSend / postRecv and :249-318 LLGenericOp), through the C ABI: two or
three "ranks" on their own streams of the one GPU, each a single call covering many steps, their FIFO
slots reused many times over (so every slot's credit comes back through the head words several times),
against numpy (two-operand sums, exact) and the oracle's LL step (oracle/nexr_oracle.c) for the fold
order of three. Also: a line or a credit that never comes ends the run within its timeout with the status
word set, and steps that touch each other's user bytes run as if one at a time."""
import ctypes

import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SLOTS = 8


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


class _OwnQueueStreams:
    """Streams with a hardware queue of their own (hipExtStreamCreateWithCUMask, every CU in the mask):
    a run waits for its peer's, so the two must not share one of HIP's GPU_MAX_HW_QUEUES queues, on
    which kernels run one after the other (the ring library makes its rank streams the same way)."""

    def __init__(self, nexr):
        self.hip = nexr.hip_runtime()
        self.hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                          ctypes.POINTER(ctypes.c_uint32)]
        self.hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
        self.hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        words = [0xFFFFFFFF] * ((cus + 31) // 32)
        if cus % 32:
            words[-1] = (1 << (cus % 32)) - 1
        self.mask = (ctypes.c_uint32 * len(words))(*words)
        self.made = []

    def __call__(self, n):
        out = []
        for _ in range(n):
            h = ctypes.c_void_p()
            assert self.hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(self.mask), self.mask) == 0
            self.made.append(h.value)
            out.append(h.value)
        return out

    def close(self):
        torch.cuda.synchronize()
        for h in self.made:
            self.hip.hipStreamDestroy(h)


@pytest.fixture(scope="module")
def streams(nexr):
    s = _OwnQueueStreams(nexr)
    yield s
    s.close()


def _conn(slot_bytes):
    """A connection's receive FIFO with its head words behind it, zeroed (as nexr_ring.cpp makes them)."""
    buf = torch.zeros(slot_bytes * SLOTS + 4096, dtype=torch.uint8, device="cuda")
    return buf, buf.data_ptr(), buf.data_ptr() + slot_bytes * SLOTS


def _status():
    return torch.zeros(1, dtype=torch.int32, device="cuda")


@pytest.mark.parametrize("slot_bytes", [4096, 1 << 16, 1 << 20])
@pytest.mark.parametrize("n_steps", [1, 9, 40])
def test_two_ranks_send_then_recv_reduce(nexr, dev, streams, slot_bytes, n_steps):
    """Rank A sends n_steps steps of its input; rank B receives each and writes peer + own input to its
    output. 4 KiB slots run one workgroup, 64 KiB eight, 1 MiB the 64-workgroup cap (each workgroup
    two tiles of every slot); 40 steps wrap the 8 slots five times. B's run is queued first, so its
    kernel polls while A's is still being queued."""
    per = slot_bytes // 2 // 4  # fp32 elements per full step
    sizes = [per - (k % 3) * 37 for k in range(n_steps)]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    total = int(offs[-1])
    rng = np.random.default_rng(slot_bytes + n_steps)
    a = rng.standard_normal(total).astype(np.float32)
    b = rng.standard_normal(total).astype(np.float32)
    da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    out = torch.zeros(total, dtype=torch.float32, device=dev)
    _keep, fifo, head = _conn(slot_bytes)
    sa, sb = streams(2)
    st_a, st_b = _status(), _status()
    torch.cuda.synchronize()
    b_steps = [nexr.ll_step(0, int(offs[k]), 1, int(offs[k]), sizes[k], recv=True) for k in range(n_steps)]
    a_steps = [nexr.ll_step(0, int(offs[k]), -1, 0, sizes[k], send=True) for k in range(n_steps)]
    nexr.reduce_copy_ll_steps(db.data_ptr(), out.data_ptr(), [(fifo, head, 0)], [], slot_bytes, b_steps, mg.F32, 0,
                              status=st_b.data_ptr(), timeout_us=5_000_000, stream=sb)
    nexr.reduce_copy_ll_steps(da.data_ptr(), 0, [], [(fifo, head, 0)], slot_bytes, a_steps, mg.F32, 0,
                              status=st_a.data_ptr(), timeout_us=5_000_000, stream=sa)
    torch.cuda.synchronize()
    assert int(st_a.item()) == 0 and int(st_b.item()) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint32), (a + b).view(np.uint32))
    # the receiver's head words (one per wave at a 16-B stride): every wave has read every step
    waves = 4 * min(64, -(-(slot_bytes // 16) // 512))
    heads = _keep[slot_bytes * SLOTS:].view(torch.int64).cpu().numpy()[::2]
    assert list(heads[:waves]) == [n_steps] * waves and not heads[waves:].any()


def test_counters_carry_over_between_runs(nexr, dev, streams):
    """Three runs in a row on the same connection, each starting at the step counters the last one
    ended at (flags step + 1 keep growing; the head words keep the credits): every element exact."""
    slot = 1 << 14
    per = slot // 2 // 4
    _keep, fifo, head = _conn(slot)
    sa, sb = streams(2)
    st = _status()
    step = 0
    for run, n in enumerate((5, 13, 21)):
        rng = np.random.default_rng(run)
        a = rng.integers(-1000, 1000, n * per).astype(np.float32)
        b = rng.integers(-1000, 1000, n * per).astype(np.float32)
        da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        out = torch.zeros_like(db)
        torch.cuda.synchronize()
        nexr.reduce_copy_ll_steps(db.data_ptr(), out.data_ptr(), [(fifo, head, step)], [], slot,
                                  [nexr.ll_step(0, k * per, 1, k * per, per, recv=True) for k in range(n)], mg.F32, 0,
                                  status=st.data_ptr(), timeout_us=5_000_000, stream=sb)
        nexr.reduce_copy_ll_steps(da.data_ptr(), 0, [], [(fifo, head, step)], slot,
                                  [nexr.ll_step(0, k * per, -1, 0, per, send=True) for k in range(n)], mg.F32, 0,
                                  status=st.data_ptr(), timeout_us=5_000_000, stream=sa)
        torch.cuda.synchronize()
        assert int(st.item()) == 0
        assert np.array_equal(out.cpu().numpy(), a + b), run
        step += n


@pytest.mark.parametrize("dt,op", [(mg.BF16, 0), (mg.F16, 1), (mg.I8, 2), (mg.F32, 4)])
def test_three_rank_chain_matches_the_oracle(nexr, oracle, dev, streams, dt, op):
    """A -> B -> C: A sends its input, B receives, folds its own input (peer first) and forwards
    (recvReduceSend), C receives, folds, applies the post-op and writes its output (recvReduceCopy) — a
    ring Reduce's chain, 30 steps over 8 slots, B both a receiver and a sender in every step."""
    slot = 1 << 15
    esz = np.dtype(mg.STORE[dt]).itemsize
    per = slot // 2 // esz
    n = 30
    total = n * per - 5
    sizes = [per] * (n - 1) + [total - (n - 1) * per]
    xs = mg.gen_inputs(dt, 3, total, 11 * dt + op, special=True)
    dev_op, arg = oracle.host_to_dev_red_op(op, dt, 3)
    dx = [torch.from_numpy(x.copy()).to(dev) for x in xs]
    out = torch.zeros_like(dx[2])
    ab, ab_fifo, ab_head = _conn(slot)
    bc, bc_fifo, bc_head = _conn(slot)
    ss = streams(3)
    st = _status()
    torch.cuda.synchronize()
    offs = [k * per for k in range(n)]
    nexr.reduce_copy_ll_steps(dx[2].data_ptr(), out.data_ptr(), [(bc_fifo, bc_head, 0)], [], slot,
                              [nexr.ll_step(0, offs[k], 1, offs[k], sizes[k], recv=True, post_op=True)
                               for k in range(n)], dt, dev_op, arg, status=st.data_ptr(), timeout_us=5_000_000,
                              stream=ss[2])
    nexr.reduce_copy_ll_steps(dx[1].data_ptr(), 0, [(ab_fifo, ab_head, 0)], [(bc_fifo, bc_head, 0)], slot,
                              [nexr.ll_step(0, offs[k], -1, 0, sizes[k], recv=True, send=True) for k in range(n)],
                              dt, dev_op, arg, status=st.data_ptr(), timeout_us=5_000_000,
                              stream=ss[1])
    nexr.reduce_copy_ll_steps(dx[0].data_ptr(), 0, [], [(ab_fifo, ab_head, 0)], slot,
                              [nexr.ll_step(0, offs[k], -1, 0, sizes[k], send=True) for k in range(n)],
                              dt, dev_op, arg, status=st.data_ptr(), timeout_us=5_000_000,
                              stream=ss[0])
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    from oracle.ring import reduce_expected
    exp = reduce_expected(xs, dt, op, 2, "ll")
    assert mg.canon_bytes(dt, out.cpu().numpy()) == mg.canon_bytes(dt, exp)


def test_a_missing_line_ends_the_run_with_status(nexr, dev, streams):
    """The receiver's peer never sends: every workgroup gives up after the timeout, sets the status
    word and ends its run (the later steps are not waited for again); the stream completes."""
    import time
    slot = 1 << 16
    _keep, fifo, head = _conn(slot)
    x = torch.ones(50 * (slot // 8), dtype=torch.float32, device=dev)
    out = torch.zeros_like(x)
    st = _status()
    (s,) = streams(1)
    torch.cuda.synchronize()
    per = slot // 8
    t0 = time.time()
    nexr.reduce_copy_ll_steps(x.data_ptr(), out.data_ptr(), [(fifo, head, 0)], [], slot,
                              [nexr.ll_step(0, k * per, 1, k * per, per, recv=True) for k in range(50)], mg.F32, 0,
                              status=st.data_ptr(), timeout_us=200_000, stream=s)
    torch.cuda.synchronize()
    dt = time.time() - t0
    assert int(st.item()) == 1
    assert dt < 5.0, dt
    assert not out.any()


def test_a_missing_credit_ends_the_run_with_status(nexr, dev, streams):
    """Nobody reads the sender's slots: 8 steps go out, the 9th waits for a credit that never comes,
    times out with the status set, and the run ends."""
    slot = 1 << 12
    per = slot // 8
    keep, fifo, head = _conn(slot)
    x = torch.arange(12 * per, dtype=torch.float32, device=dev)
    st = _status()
    (s,) = streams(1)
    torch.cuda.synchronize()
    nexr.reduce_copy_ll_steps(x.data_ptr(), 0, [], [(fifo, head, 0)], slot,
                              [nexr.ll_step(0, k * per, -1, 0, per, send=True) for k in range(12)], mg.F32, 0,
                              status=st.data_ptr(), timeout_us=200_000, stream=s)
    torch.cuda.synchronize()
    assert int(st.item()) == 1
    lines = keep[:slot * SLOTS].cpu().numpy().view(np.uint32).reshape(-1, 4)
    # slots 0-7 hold steps 1-8 (flags 1..8); step 9 was never written over slot 0
    flags = lines[:, 1].reshape(SLOTS, -1)
    assert [int(f[0]) for f in flags] == list(range(1, 9))
    first = x[:per].cpu().numpy()
    assert np.array_equal(lines[: slot // 16, 0].view(np.float32), first[0::2])
    assert np.array_equal(lines[: slot // 16, 2].view(np.float32), first[1::2])


def test_overlapping_user_ranges_run_as_if_one_at_a_time(nexr, dev):
    """Copies within the user buffers, no connections: step k reads output[P(k-1) + 13 : + n] and writes
    output[P(k)] with P(k) = (k % 2) * 20000, so every step reads what the one before wrote at another
    position (and writes what the one before that read at another position) — the library starts a new
    launch for each; and 40 in-place scalings of one range (the same range at the same position: one
    launch) — both exact against the sequential result."""
    n, off, d = 5000, 20000, 13
    x = np.random.default_rng(3).integers(-100, 100, n).astype(np.float32)
    total = 2 * off
    out = torch.zeros(total, dtype=torch.float32, device=dev)
    din = torch.from_numpy(x).to(dev)
    st = _status()
    steps = [nexr.ll_step(0, 0, 1, 0, n)] + [nexr.ll_step(1, ((k - 1) % 2) * off + d, 1, (k % 2) * off, n)
                                             for k in range(1, 11)]
    torch.cuda.synchronize()
    nexr.reduce_copy_ll_steps(din.data_ptr(), out.data_ptr(), [], [], 1 << 16, steps, mg.F32, 0,
                              status=st.data_ptr())
    torch.cuda.synchronize()
    exp = np.zeros(total, np.float32)
    exp[:n] = x
    for k in range(1, 11):
        src = ((k - 1) % 2) * off + d
        exp[(k % 2) * off:(k % 2) * off + n] = exp[src:src + n].copy()
    assert np.array_equal(out.cpu().numpy(), exp)
    two = int(np.float32(2.0).view(np.uint32))
    y = torch.from_numpy(x.copy()).to(dev)
    torch.cuda.synchronize()
    # PreMulSum with the input as source scales by the scalar: input *= 2, forty times, in place
    nexr.reduce_copy_ll_steps(y.data_ptr(), 0, [], [], 1 << 16, [nexr.ll_step(0, 0, 0, 0, n)] * 40, mg.F32, 3,
                              two, status=st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert np.array_equal(y.cpu().numpy(), x * np.float32(2.0 ** 40))


def test_a_host_abort_ends_the_run(nexr, dev, streams):
    """The status word as an abort flag (checkAbort, primitives.h:142-156): a run waiting for lines that
    never come, with a 10 s timeout, ends soon after the host writes 2 into its (pinned, device-mapped)
    status word — the ring's rank threads relay another rank's failure this way."""
    import time
    slot = 1 << 16
    per = slot // 8
    _keep, fifo, head = _conn(slot)
    x = torch.ones(20 * per, dtype=torch.float32, device=dev)
    out = torch.zeros_like(x)
    st = torch.zeros(1, dtype=torch.int32).pin_memory()
    (s,) = streams(1)
    torch.cuda.synchronize()
    t0 = time.time()
    nexr.reduce_copy_ll_steps(x.data_ptr(), out.data_ptr(), [(fifo, head, 0)], [], slot,
                              [nexr.ll_step(0, k * per, 1, k * per, per, recv=True) for k in range(20)], mg.F32, 0,
                              status=st.data_ptr(), timeout_us=10_000_000, stream=s)
    time.sleep(0.2)
    st[0] = 2
    torch.cuda.synchronize()
    assert time.time() - t0 < 3.0
    assert int(st[0]) == 2 and not out.any()
