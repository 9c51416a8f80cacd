"""LL / LL128 flag protocol under real concurrency.

The emulated collectives launch a receiver's step only after the sender's (the host waits on the
tail counter, nexr_emu.h genericOpLL), so their GPU tests see line flags either already valid or
never valid. Here the receiver's kernel is launched FIRST, on its own stream, and polls the FIFO
lines while the sender's kernel — launched after it on a second stream — is still writing them: the
receiver reads lines whose flags flip under it, exactly the situation the protocols exist for
(prims_ll.h:91-109 readLL, prims_ll128.h:200-265 recvReduceSendCopy with the per-line flag word).
Every step reuses the same wire buffer with the next flag value, as a FIFO slot is reused. Outputs
are checked bit-exactly (the receiver folds peer first: out = op(peer, x)); a receiver that accepted
a line before its data landed would show up as a mismatch, and one that never saw the flag as a
status/timeout.
"""
import ctypes

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _ll_wire_bytes(n_bytes):
    return ((n_bytes + 7) // 8) * 16 + 64


def _ll128_wire_bytes(n_bytes):
    return -(-n_bytes // 1920) * 2048 + 64


@pytest.mark.parametrize("proto", ["ll", "ll128"])
@pytest.mark.parametrize("dtype,n", [(torch.int32, 131_072), (torch.float32, 262_139), (torch.int32, 1_000_003)])
def test_receiver_polls_while_sender_writes(nexr, proto, dtype, n):
    dev = torch.device("cuda")
    dt = nexr.torch_datatype(dtype)
    esz = torch.empty((), dtype=dtype).element_size()
    wire_bytes = (_ll_wire_bytes if proto == "ll" else _ll128_wire_bytes)(n * esz)
    wire = torch.zeros(wire_bytes, dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    # Two HIP streams created back to back land on different hardware queues (HIP assigns queues
    # round-robin at creation, GPU_MAX_HW_QUEUES = 4), so the sender can run beside the polling
    # receiver. (torch's pooled streams may share one queue: the sender would then wait behind a
    # receiver that waits for it, until the receiver's bounded poll times out.)
    hip = nexr.hip_runtime()
    handles = []
    for _ in range(2):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0  # hipStreamNonBlocking
        handles.append(h)
    s_recv, s_send = (torch.cuda.ExternalStream(h.value) for h in handles)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    run = nexr.reduce_copy_ll if proto == "ll" else nexr.reduce_copy_ll128
    steps, bad, overlapped = 40, [], 0
    for step in range(1, steps + 1):
        if dtype == torch.int32:
            x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=dtype, device=dev, generator=g)
            y = torch.randint(-2**31, 2**31 - 1, (n,), dtype=dtype, device=dev, generator=g)
            expect = (y.to(torch.int64) + x.to(torch.int64)).to(torch.int32)  # wraps like the uint32 kernel
        else:
            x = torch.rand(n, device=dev, generator=g) * 2 - 1
            y = torch.rand(n, device=dev, generator=g) * 2 - 1
            expect = y + x
        out = torch.full_like(x, -1)
        flag = step if proto == "ll" else (1 << 33) + step
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        # receiver first: recv(peer) + local x -> out, polling the wire
        ev[0].record(s_recv)
        run(x.data_ptr(), [wire.data_ptr()], [flag], out.data_ptr(), [], [], n, dt, 0, 0, True, False,
            status=status.data_ptr(), timeout_us=2_000_000, stream=s_recv.cuda_stream)
        ev[2].record(s_recv)
        # then the sender: y -> wire with this step's flag
        ev[1].record(s_send)
        run(y.data_ptr(), [], [], 0, [wire.data_ptr()], [flag], n, dt, 0, 0, True, False,
            stream=s_send.cuda_stream)
        s_send.synchronize()
        s_recv.synchronize()
        # the receiver's kernel was on the GPU before the sender's started and ended after it started:
        # it polled lines the sender had not written yet
        if ev[0].elapsed_time(ev[1]) > 0 and ev[1].elapsed_time(ev[2]) > 0:
            overlapped += 1
        assert int(status.item()) == 0, f"step {step}: receiver timed out"
        if not torch.equal(out.view(torch.int32), expect.view(torch.int32)):
            bad.append((step, int((out.view(torch.int32) != expect.view(torch.int32)).sum())))
    for h in handles:
        assert hip.hipStreamDestroy(h) == 0
    assert not bad, f"{proto}: steps with elements taken before their data landed: {bad}"
    assert overlapped >= steps // 2, f"only {overlapped} of {steps} steps ran the receiver beside the sender"
    print(f"{proto} n={n}: {overlapped}/{steps} steps with the receiver polling while the sender wrote")
