"""GPU tests of ncclSend/ncclRecv on the emulated communicator (nexrSendRecv) with the MI355X
reduce-copy doing every chunk copy: buffers and connection-index-1 FIFOs in HBM (the send half on
the rank's stream, the recv half on its second stream) and in host memory (nexrReduceCopyHost)."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ring(nexr):
    assert torch.cuda.is_available()
    from conftest import extras_ring
    return extras_ring()  # include/nexr_extras.h: skipped when the opt-in library is not built


@pytest.mark.parametrize("n,shift,nbytes,buff", [(2, 1, 3_000_001, 0), (4, 1, 1 << 20, 1 << 16), (5, 2, 77_777, 1 << 15),
                                                 (8, 3, 1 << 22, 0), (3, 0, 123_457, 0),
                                                 # <= 16 KiB: the LL protocol (nexrReduceCopyLL steps)
                                                 (2, 1, 1, 0), (3, 1, 4_097, 0), (4, 3, 16_384, 1 << 16)])
def test_send_recv_device(ring, n, shift, nbytes, buff):
    g = torch.Generator(device="cuda")
    g.manual_seed(n * 7 + shift)
    send = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(n)]
    recv = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()
    sp = [(r + shift) % n for r in range(n)]
    rp = [(r - shift) % n for r in range(n)]
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff) as comm:
        for _ in range(2):  # links and their step counters persist between calls
            comm.send_recv([t.data_ptr() for t in send], sp, [t.data_ptr() for t in recv], rp, nbytes)
            for r in range(n):
                assert torch.equal(recv[r], send[rp[r]]), r
            send = send[1:] + send[:1]


def test_send_recv_host_memory(ring):
    n, nbytes = 4, 500_003
    rng = np.random.default_rng(3)
    send = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
    recv = [np.zeros(nbytes, np.uint8) for _ in range(n)]
    with ring.RingComm(n, ring.HOST_MEMORY, 1 << 16) as comm:
        comm.send_recv([s.ctypes.data for s in send], [r ^ 1 for r in range(n)], [r.ctypes.data for r in recv],
                       [r ^ 1 for r in range(n)], nbytes)
    for r in range(n):
        assert recv[r].tobytes() == send[r ^ 1].tobytes()
