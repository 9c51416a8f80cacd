"""GPU parity of the LL-protocol step (nexrReduceCopyLL) against the oracle's LL restatement:
every datatype x op x the LLGenericOp shapes the collectives use (send, recvReduceSend,
recvReduceCopySend, recvCopySend, recv, two peers), odd sizes (partial last line, odd line count),
misaligned user buffers, and the bounded wait when a flag never arrives (status word, no hang)."""
import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SHAPES = {  # name: (has src, nRecv, has dst, nSend) — prims_ll.h:325-419 wrappers
    "send": (1, 0, 0, 1), "recvReduceSend": (1, 1, 0, 1), "recvReduceCopySend": (1, 1, 1, 1),
    "recvCopySend": (0, 1, 1, 1), "recv": (0, 1, 1, 0), "twoPeers": (1, 2, 1, 2), "copy": (1, 0, 1, 0),
}


def _dev(a: np.ndarray, off: int = 0):
    raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(raw.size + off + 64, dtype=torch.uint8, device="cuda")
    if raw.size:
        t[off:off + raw.size] = torch.from_numpy(raw.copy()).cuda()
    return t


def _run(nexr, oracle, dt, op, arg, post, shape, n, src_off=0, dst_off=0, seed=0):
    has_src, n_recv, has_dst, n_send = SHAPES[shape]
    esz = np.dtype(mg.STORE[dt]).itemsize
    bufs = mg.gen_inputs(dt, 1 + n_recv, n, 1234 + seed, special=True)
    src = bufs[0] if has_src else None
    rflags = [100 + i for i in range(n_recv)]
    sflags = [200 + i for i in range(n_send)]
    rlines = [oracle.make_ll_lines(bufs[1 + i], rflags[i]) for i in range(n_recv)]
    rc, odst, osends = oracle.reduce_copy_ll(src, True, rlines, rflags, bool(has_dst), n_send, sflags, n, dt, op, arg,
                                             post)
    assert rc == 0
    d_src = _dev(src, src_off) if has_src else None
    d_recv = [_dev(l) for l in rlines]
    n_lines = (n * esz + 7) // 8
    d_dst = torch.full((n * esz + dst_off + 64,), 0x5A, dtype=torch.uint8, device="cuda") if has_dst else None
    d_send = [torch.zeros(n_lines * 16 + 64, dtype=torch.uint8, device="cuda") for _ in range(n_send)]
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nexr.reduce_copy_ll(d_src.data_ptr() + src_off if has_src else 0, [t.data_ptr() for t in d_recv], rflags,
                        d_dst.data_ptr() + dst_off if has_dst else 0, [t.data_ptr() for t in d_send], sflags, n, dt,
                        op, arg, True, post, status=status.data_ptr(), timeout_us=2_000_000,
                        stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    if has_dst:
        h = d_dst.cpu().numpy()
        got = h[dst_off:dst_off + n * esz].view(mg.STORE[dt])
        assert (h[:dst_off] == 0x5A).all() and (h[dst_off + n * esz:] == 0x5A).all()
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, odst.view(mg.STORE[dt]))
    for t, o in zip(d_send, osends):
        g = t.cpu().numpy()[:n_lines * 16].view(np.uint32).reshape(-1, 4)
        e = o.view(np.uint32).reshape(-1, 4)
        assert (g[:, 1] == e[:, 1]).all() and (g[:, 3] == e[:, 3]).all()          # flags
        gd = np.stack([g[:, 0], g[:, 2]], 1).reshape(-1).view(np.uint8)[:n * esz]  # valid data bytes
        ed = np.stack([e[:, 0], e[:, 2]], 1).reshape(-1).view(np.uint8)[:n * esz]
        assert mg.canon_bytes(dt, gd.view(mg.STORE[dt])) == mg.canon_bytes(dt, ed.view(mg.STORE[dt]))


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_ll_all_ops_and_shapes(nexr, oracle, dt):
    ops = [("sum", mg.SUM, 0, False), ("prod", mg.PROD, 0, False),
           ("min", mg.MINMAX, mg.minmax_arg(dt, False), False), ("max", mg.MINMAX, mg.minmax_arg(dt, True), False),
           ("premulsum", mg.PREMULSUM, mg.float_scalar_bits(dt, 0.5 if dt not in mg.INTS else 3), False)]
    if dt in mg.INTS:
        ops.append(("sumpostdiv", mg.SUMPOSTDIV, (3 << 1) | int(dt in (mg.I8, mg.I32, mg.I64)), True))
    for k, (name, op, arg, post) in enumerate(ops):
        for j, shape in enumerate(SHAPES):
            for n in (1, 3, 1001):
                _run(nexr, oracle, dt, op, arg, post, shape, n, seed=k * 100 + j * 10 + n)


def test_ll_large_and_misaligned(nexr, oracle):
    _run(nexr, oracle, mg.BF16, mg.SUM, 0, False, "recvReduceCopySend", 1_000_003, seed=9)
    _run(nexr, oracle, mg.F32, mg.SUM, 0, False, "recvReduceCopySend", 70_001, src_off=4, dst_off=12, seed=10)
    _run(nexr, oracle, mg.I8, mg.MINMAX, mg.minmax_arg(mg.I8, True), False, "twoPeers", 50_001, src_off=3, dst_off=5)


def test_ll_missing_flag_times_out_without_hanging(nexr, oracle):
    n = 4096
    data = mg.gen_inputs(mg.F32, 2, n, 3, False)
    line = _dev(oracle.make_ll_lines(data[1], 41))          # carries flag 41
    src = _dev(data[0])
    dst = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nexr.reduce_copy_ll(src.data_ptr(), [line.data_ptr()], [42], dst.data_ptr(), [], [], n, mg.F32, mg.SUM,
                        status=status.data_ptr(), timeout_us=2000, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(status.item()) == 1
    assert int(dst.count_nonzero()) == 0  # nothing written for lines that never became valid


def test_ll_tile_boundaries(nexr, oracle):
    """Sizes around the kernel's layout: a wave's 128 lines (lanes j and j + 64), a tile's 512 lines,
    and partial last lines, on int8 (byte-granular sizes) and fp32, misaligned user buffers too."""
    for k, lines in enumerate((63, 64, 65, 127, 128, 129, 511, 512, 513, 1025)):
        for extra in (-3, 0):
            n = lines * 8 + extra
            _run(nexr, oracle, mg.I8, mg.SUM, 0, False, "recvReduceCopySend", n, src_off=k % 3, dst_off=1, seed=k)
        _run(nexr, oracle, mg.F32, mg.MINMAX, mg.minmax_arg(mg.F32, True), False, "twoPeers", lines * 2 - 1,
             seed=50 + k)


def test_ll_beyond_the_grid_cap(nexr):
    """The launch caps the grid at 2^20 tiles of 512 lines (4 GiB of data) and the kernel strides
    over the rest: a 4 GiB + 12,345-byte uint8 step, its wire written by a send step and then reduced
    with a local buffer (dst = peer + src, checked against torch)."""
    n = (1 << 32) + 12_345
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    peer = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    wire = torch.zeros(((n + 7) // 8) * 16, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    nexr.reduce_copy_ll(peer.data_ptr(), [], [], 0, [wire.data_ptr()], [77], n, mg.U8, mg.SUM, stream=s)
    del peer
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.empty_like(src)
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nexr.reduce_copy_ll(src.data_ptr(), [wire.data_ptr()], [77], dst.data_ptr(), [], [], n, mg.U8, mg.SUM,
                        status=status.data_ptr(), timeout_us=2_000_000, stream=s)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    g.manual_seed(3)
    peer = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    assert torch.equal(dst, peer + src)
    del peer, wire, src, dst
    torch.cuda.empty_cache()
