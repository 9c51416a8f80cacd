"""GPU parity of the LL128-protocol step (nexrReduceCopyLL128) against the oracle's literal
warp-32 restatement: every datatype x op x step shape, partial slices, misaligned user buffers, and
the bounded wait on a stale line flag."""
import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SHAPES = {"send": (1, 0, 0, 1), "recvReduceSend": (1, 1, 0, 1), "recvReduceCopySend": (1, 1, 1, 1),
          "recvCopySend": (0, 1, 1, 1), "recv": (0, 1, 1, 0), "twoPeers": (1, 2, 1, 2), "copy": (1, 0, 1, 0)}


def _dev(a, off=0):
    raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(raw.size + off + 64, dtype=torch.uint8, device="cuda")
    if raw.size:
        t[off:off + raw.size] = torch.from_numpy(raw.copy()).cuda()
    return t


def _run(nexr, oracle, dt, op, arg, post, shape, n, src_off=0, dst_off=0, seed=0):
    has_src, n_recv, has_dst, n_send = SHAPES[shape]
    esz = np.dtype(mg.STORE[dt]).itemsize
    bufs = mg.gen_inputs(dt, 1 + n_recv, n, 4321 + seed, special=True)
    src = bufs[0] if has_src else None
    rflags = [1000 + i for i in range(n_recv)]
    sflags = [(1 << 40) + i for i in range(n_send)]
    wires = [oracle.make_ll128_wire(bufs[1 + i], rflags[i], dt) for i in range(n_recv)]
    rc, odst, osends = oracle.reduce_copy_ll128(src, True, wires, rflags, bool(has_dst), n_send, sflags, n, dt, op,
                                                arg, post)
    assert rc == 0
    n_slices = -(-(n * esz) // 1920)
    d_src = _dev(src, src_off) if has_src else None
    d_recv = [_dev(w) for w in wires]
    d_dst = torch.full((n * esz + dst_off + 64,), 0x5A, dtype=torch.uint8, device="cuda") if has_dst else None
    d_send = [torch.zeros(n_slices * 2048 + 64, dtype=torch.uint8, device="cuda") for _ in range(n_send)]
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nexr.reduce_copy_ll128(d_src.data_ptr() + src_off if has_src else 0, [t.data_ptr() for t in d_recv], rflags,
                           d_dst.data_ptr() + dst_off if has_dst else 0, [t.data_ptr() for t in d_send], sflags, n,
                           dt, op, arg, True, post, status=status.data_ptr(), timeout_us=2_000_000,
                           stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    if has_dst:
        h = d_dst.cpu().numpy()
        assert (h[:dst_off] == 0x5A).all() and (h[dst_off + n * esz:] == 0x5A).all()
        assert mg.canon_bytes(dt, h[dst_off:dst_off + n * esz].view(mg.STORE[dt])) == \
            mg.canon_bytes(dt, odst.view(mg.STORE[dt]))
    for t, o in zip(d_send, osends):
        g = t.cpu().numpy()[:n_slices * 2048].view(np.uint64).reshape(-1, 16)
        e = o.view(np.uint64).reshape(-1, 16)
        assert (g[:, 15] == e[:, 15]).all()  # flags
        # decode both wires with the oracle (recv-only) and compare the valid data
        _, gd, _ = oracle.reduce_copy_ll128(None, False, [g.reshape(-1).view(np.uint8).copy()], [int(e[0, 15])], True,
                                            0, [], n, dt, mg.SUM)
        _, ed, _ = oracle.reduce_copy_ll128(None, False, [o], [int(e[0, 15])], True, 0, [], n, dt, mg.SUM)
        assert mg.canon_bytes(dt, gd.view(mg.STORE[dt])) == mg.canon_bytes(dt, ed.view(mg.STORE[dt]))


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_ll128_all_ops_and_shapes(nexr, oracle, dt):
    ops = [("sum", mg.SUM, 0, False), ("prod", mg.PROD, 0, False),
           ("min", mg.MINMAX, mg.minmax_arg(dt, False), False), ("max", mg.MINMAX, mg.minmax_arg(dt, True), False),
           ("premulsum", mg.PREMULSUM, mg.float_scalar_bits(dt, 0.5 if dt not in mg.INTS else 3), False)]
    if dt in mg.INTS:
        ops.append(("sumpostdiv", mg.SUMPOSTDIV, (3 << 1) | int(dt in (mg.I8, mg.I32, mg.I64)), True))
    for k, (name, op, arg, post) in enumerate(ops):
        for j, shape in enumerate(SHAPES):
            for n in (1, 3, 5000):
                _run(nexr, oracle, dt, op, arg, post, shape, n, seed=k * 100 + j * 10 + n % 7)


def test_ll128_large_and_misaligned(nexr, oracle):
    _run(nexr, oracle, mg.BF16, mg.SUM, 0, False, "recvReduceCopySend", 1_000_003, seed=1)
    _run(nexr, oracle, mg.F32, mg.SUM, 0, False, "recvReduceCopySend", 70_001, src_off=4, dst_off=12, seed=2)
    _run(nexr, oracle, mg.I8, mg.MINMAX, mg.minmax_arg(mg.I8, False), False, "twoPeers", 50_001, src_off=3, dst_off=9)


def test_ll128_stale_flag_times_out(nexr, oracle):
    n = 4000
    x = mg.gen_inputs(mg.F32, 2, n, 8, False)
    wire = oracle.make_ll128_wire(x[1], 9, mg.F32)
    wire.view(np.uint64).reshape(-1, 16)[3, 15] = 8
    dst = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nexr.reduce_copy_ll128(_dev(x[0]).data_ptr(), [_dev(wire).data_ptr()], [9], dst.data_ptr(), [], [], n, mg.F32,
                           mg.SUM, status=status.data_ptr(), timeout_us=2000,
                           stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(status.item()) == 1


def test_ll128_tile_boundaries(nexr, oracle):
    """Sizes around the kernel's layout: one 1920-byte slice, a tile's two slices (3840 bytes), and
    partial last lines and chunks, on int8 (byte-granular sizes) and fp32, misaligned user buffers too."""
    for k, n in enumerate((1919, 1920, 1921, 1928, 3839, 3840, 3841, 5760, 7681)):
        _run(nexr, oracle, mg.I8, mg.SUM, 0, False, "recvReduceCopySend", n, src_off=k % 3, dst_off=1, seed=k)
        _run(nexr, oracle, mg.F32, mg.PROD, 0, False, "twoPeers", -(-n // 4), seed=50 + k)


def test_ll128_beyond_the_grid_cap(nexr):
    """The launch caps the grid at 2^20 tiles of two slices (3,840 data bytes each) and the kernel
    strides over the rest: a 2^32 + 12,345-byte uint8 step (past the cap), its wire written by a send
    step and then reduced with a local buffer (dst = peer + src, checked against torch)."""
    n = (1 << 32) + 12_345
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    peer = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    wire = torch.zeros(-(-n // 1920) * 2048, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    nexr.reduce_copy_ll128(peer.data_ptr(), [], [], 0, [wire.data_ptr()], [(1 << 40) + 5], n, mg.U8, mg.SUM, stream=s)
    del peer
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.empty_like(src)
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nexr.reduce_copy_ll128(src.data_ptr(), [wire.data_ptr()], [(1 << 40) + 5], dst.data_ptr(), [], [], n, mg.U8,
                           mg.SUM, status=status.data_ptr(), timeout_us=2_000_000, stream=s)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    g.manual_seed(4)
    peer = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    assert torch.equal(dst, peer + src)
    del peer, wire, src, dst
    torch.cuda.empty_cache()
