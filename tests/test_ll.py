"""CPU tests of the LL-protocol step (LLGenericOp, reference src/device/prims_ll.h:218-283) in the
oracle: wire format of ncclLLFifoLine (device.h:695-708), the peer-FIRST operand order of
applyReduce(redOp, peerData, data), pre-op on the user input, post-op, partial last line, and the
not-ready case when a flag does not match."""
import numpy as np
import pytest

import make_golden as mg


def test_line_encoding_matches_ncclLLFifoLine(oracle):
    data = np.arange(1, 6, dtype=np.uint32)  # 20 bytes -> 3 lines
    lines = oracle.make_ll_lines(data, 0xABC).view(np.uint32).reshape(-1, 4)
    assert lines.tolist() == [[1, 0xABC, 2, 0xABC], [3, 0xABC, 4, 0xABC], [5, 0xABC, 0, 0xABC]]


@pytest.mark.parametrize("dt,name", [(mg.F32, "sum"), (mg.I32, "min"), (mg.BF16, "max"), (mg.U8, "prod"),
                                     (mg.F64, "sum"), (mg.F16, "min")])
def test_ll_recv_reduce_is_peer_first(oracle, dt, name):
    n = 1003
    op = {"sum": mg.SUM, "prod": mg.PROD, "min": mg.MINMAX, "max": mg.MINMAX}[name]
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    local, p0, p1 = mg.gen_inputs(dt, 3, n, 70 + dt, special=True)
    lines = [oracle.make_ll_lines(p0, 7), oracle.make_ll_lines(p1, 9)]
    rc, dst, sends = oracle.reduce_copy_ll(local, True, lines, [7, 9], True, 1, [11], n, dt, op, arg)
    assert rc == 0
    # d = op(peer1, op(peer0, local)): two left folds with the peer as the accumulator
    step1 = oracle.reduce_copy([p0, local], 1, dt, op, arg)[0]
    exp = oracle.reduce_copy([p1, step1], 1, dt, op, arg)[0]
    assert mg.canon_bytes(dt, dst.view(exp.dtype)) == mg.canon_bytes(dt, exp)
    sent = sends[0].view(np.uint32).reshape(-1, 4)
    assert (sent[:, 1] == 11).all() and (sent[:, 3] == 11).all()
    data = np.stack([sent[:, 0], sent[:, 2]], axis=1).reshape(-1).view(np.uint8)[:n * exp.itemsize]
    assert mg.canon_bytes(dt, data.view(exp.dtype)) == mg.canon_bytes(dt, exp)


def test_ll_send_only_applies_preop_and_recv_only_copies(oracle):
    n = 77
    x = mg.gen_inputs(mg.F32, 1, n, 5, False)[0]
    half = mg.float_scalar_bits(mg.F32, 0.5)
    rc, _, sends = oracle.reduce_copy_ll(x, True, [], [], False, 1, [3], n, mg.F32, mg.PREMULSUM, half)
    assert rc == 0
    sent = sends[0].view(np.uint32).reshape(-1, 4)
    got = np.stack([sent[:, 0], sent[:, 2]], axis=1).reshape(-1).view(np.float32)[:n]
    assert np.array_equal(got, (x * np.float32(0.5)).astype(np.float32))
    # recv-only: d = peer (no arithmetic, NaN payload survives)
    h = np.array([0x7E01, 0x3C00, 0x0001], dtype=np.uint16)
    rc, dst, _ = oracle.reduce_copy_ll(None, False, [oracle.make_ll_lines(h, 1)], [1], True, 0, [], 3, mg.F16, mg.SUM)
    assert rc == 0 and dst.view(np.uint16).tolist() == h.tolist()


def test_ll_postop_divides_and_flag_mismatch_is_not_ready(oracle):
    n = 9
    a = np.array([10, -10, 7, -7, 100, 0, 1, -1, 5], dtype=np.int32)
    b = np.array([2, -2, 0, 0, 100, 0, 1, -1, 5], dtype=np.int32)
    arg = (2 << 1) | 1  # Avg over 2 ranks, signed
    rc, dst, _ = oracle.reduce_copy_ll(a, True, [oracle.make_ll_lines(b, 4)], [4], True, 0, [], n, mg.I32,
                                       mg.SUMPOSTDIV, arg, post_op=True)
    assert rc == 0
    assert dst.view(np.int32).tolist() == [int((x + y) / 2) for x, y in zip(a.tolist(), b.tolist())]
    rc, _, _ = oracle.reduce_copy_ll(a, True, [oracle.make_ll_lines(b, 4)], [5], True, 0, [], n, mg.I32, mg.SUM)
    assert rc == 3
