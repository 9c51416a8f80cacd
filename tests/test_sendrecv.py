"""CPU tests of ncclSend/ncclRecv on the emulated communicator (nexrSendRecv; the P2P work batch of
reference src/device/sendrecv.h): every rank's send beside its recv, chunked through 8-step FIFOs of
the P2P chunk size, self-sends as one copy. A copy has one right answer: recvbuffs[r] must equal
the bytes of sendbuffs[recvPeers[r]]. The oracle serves every reduceCopy (K = 1 copies)."""
import ctypes
import importlib

import numpy as np
import pytest


@pytest.fixture(scope="module")
def ring(nexr):
    from conftest import extras_ring
    return extras_ring()  # include/nexr_extras.h: skipped when the opt-in library is not built


@pytest.fixture(scope="module")
def fn(oracle):
    return ctypes.cast(oracle.lib().oracle_reduce_copy_fn, ctypes.c_void_p).value


def _run(ring, fn, n, send_peers, recv_peers, nbytes, buff=8 * 1024, comm=None, seed=0):
    rng = np.random.default_rng(seed)
    send = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
    recv = [np.zeros(nbytes, np.uint8) for _ in range(n)]
    own = comm is None
    comm = comm or ring.RingComm(n, ring.HOST_MEMORY, buff, fn, 20000)
    try:
        comm.send_recv([s.ctypes.data for s in send], send_peers, [r.ctypes.data for r in recv], recv_peers, nbytes)
    finally:
        if own:
            comm.close()
    for r in range(n):
        if recv_peers[r] >= 0:
            assert recv[r].tobytes() == send[recv_peers[r]].tobytes(), r
        else:
            assert not recv[r].any(), r
    return send, recv


@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("nbytes", [1, 17, 1024, 1025, 50_001])  # 50 KB > 8 steps of 1 KiB: FIFO wrap
def test_ring_shift(ring, fn, n, nbytes):
    _run(ring, fn, n, [(r + 1) % n for r in range(n)], [(r - 1) % n for r in range(n)], nbytes, seed=n * nbytes)


@pytest.mark.parametrize("n", [2, 4, 6])
def test_pairwise_exchange_and_self(ring, fn, n):
    _run(ring, fn, n, [r ^ 1 for r in range(n)], [r ^ 1 for r in range(n)], 33_333)
    _run(ring, fn, n, list(range(n)), list(range(n)), 12_345)  # every rank to itself


def test_partial_participation_and_all_to_all_by_shifts(ring, fn):
    n = 5
    # only 1 -> 3 and 4 -> 4 (self) move
    _run(ring, fn, n, [-1, 3, -1, -1, 4], [-1, -1, -1, 1, 4], 9_000)
    # an all-to-all as n-1 grouped shifts on one communicator (links persist between calls)
    with ring.RingComm(n, ring.HOST_MEMORY, 8 * 1024, fn, 20000) as comm:
        for k in range(1, n):
            _run(ring, fn, n, [(r + k) % n for r in range(n)], [(r - k) % n for r in range(n)], 7_777 + k,
                 comm=comm, seed=k)
        # and the ring collectives still run on the same communicator
        x = [np.full(4000, r + 1, np.float32) for r in range(n)]
        out = [np.zeros_like(v) for v in x]
        comm.all_reduce([v.ctypes.data for v in x], [v.ctypes.data for v in out], 4000, 7, 0)
        assert all(np.all(o == sum(range(1, n + 1))) for o in out)


def test_send_recv_rejects_unmatched(ring, fn, nexr):
    a = np.zeros(64, np.uint8)
    ptrs = [a.ctypes.data] * 3
    with ring.RingComm(3, ring.HOST_MEMORY, 8 * 1024, fn, 20000) as comm:
        with pytest.raises(nexr.NexrError):
            comm.send_recv(ptrs, [1, -1, -1], ptrs, [-1, -1, -1], 64)  # 0 -> 1 but 1 does not recv
        with pytest.raises(nexr.NexrError):
            comm.send_recv(ptrs, [1, 2, 0], ptrs, [1, 2, 0], 64)  # 0 expects 1's message, but 1 sends to 2
        with pytest.raises(nexr.NexrError):
            comm.send_recv(ptrs, [3, -1, -1], ptrs, [-1, -1, -1], 64)  # peer out of range
        comm.send_recv(ptrs, [-1] * 3, ptrs, [-1] * 3, 64)  # nothing to do
        comm.send_recv(ptrs, [1, 2, 0], ptrs, [2, 0, 1], 0)  # empty messages
    with ring.RingComm(2, ring.HOST_MEMORY, 8 * 1024, fn, 20000, ring.PROTO_LL, fn, fn) as comm:
        with pytest.raises(nexr.NexrError):
            comm.send_recv(ptrs[:2], [1, 0], ptrs[:2], [1, 0], 64)


_LL_ARGS = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
            ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
LL_CALLS = []


@pytest.fixture(scope="module")
def ll_fn(oracle):
    """The oracle's LL step behind a counting trampoline (nexrReduceCopyLLFn signature)."""
    target = oracle.lib().oracle_reduce_copy_ll_fn
    target.argtypes, target.restype = _LL_ARGS, ctypes.c_int
    proto = ctypes.CFUNCTYPE(ctypes.c_int, *_LL_ARGS)

    def tramp(*args):
        LL_CALLS.append(args[9])  # nElts of the step
        return target(*args)

    cb = proto(tramp)
    ll_fn.keep = cb  # keep the trampoline alive for the module
    return ctypes.cast(cb, ctypes.c_void_p).value


@pytest.mark.parametrize("nbytes", [1, 8, 15, 1000, 16_384, 16_385, 40_000])
def test_small_messages_take_ll(ring, fn, ll_fn, nbytes):
    """Messages up to 16 KiB travel as LL lines (NCCL_P2P_LL_THRESHOLD, enqueue.cc:786-839) when an LL
    step implementation is available (here the oracle's); larger ones as SIMPLE chunks. Both kinds of
    link persist on one communicator, with self-sends (plain copies) in between."""
    n = 4
    LL_CALLS.clear()
    with ring.RingComm(n, ring.HOST_MEMORY, 8 * 1024, fn, 20000, ring.PROTO_SIMPLE, ll_fn) as comm:
        for it, shift in enumerate((1, 3, 0, 2, 1)):
            _run(ring, fn, n, [(r + shift) % n for r in range(n)], [(r - shift) % n for r in range(n)],
                 nbytes if it % 2 == 0 else 20_000, comm=comm, seed=it)
    # calls 0 and 4 move `nbytes` between distinct ranks (call 2 is a self-send): one LL step per
    # send and per recv, each carrying the whole message
    expect = 2 * 2 * n if nbytes <= 16_384 else 0
    assert len(LL_CALLS) == expect and all(v == nbytes for v in LL_CALLS)
