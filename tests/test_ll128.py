"""CPU tests of the LL128 step restatement (oracle_reduce_copy_ll128, a literal restatement of the
reference's warp-32 register flow in src/device/prims_ll128.h:86-331).

The wire layout is cross-checked against an independent per-16-byte-unit formulation (the one the
gfx950 kernel uses): unit q = 32g + w of a 2 KiB slice carries user chunk
ix = g*32 - 4*(g/2) + w - (g%2)*(w/8), except w % 8 == 7 units, which carry one 8-byte half of chunk
ix(g & ~1, w) and the line flag."""
import numpy as np
import pytest

import make_golden as mg


def unit_map():
    """(q -> (data byte offset within the slice, length)) per the unit formulation."""
    m = []
    for q in range(128):
        g, w = q // 32, q % 32
        if w % 8 != 7:
            m.append(((g * 32 - 4 * (g // 2) + w - (g % 2) * (w // 8)) * 16, 16))
        else:
            ge = g & ~1
            m.append(((ge * 32 - 4 * (ge // 2) + w) * 16 + (g & 1) * 8, 8))
    return m


def test_unit_map_is_a_partition_of_the_1920_data_bytes():
    covered = np.zeros(1920, dtype=int)
    for off, ln in unit_map():
        covered[off:off + ln] += 1
    assert (covered == 1).all()


@pytest.mark.parametrize("n_bytes", [1920, 3840, 1921, 100, 7 * 1920 + 1000])
def test_oracle_wire_matches_unit_formulation(oracle, n_bytes):
    data = np.random.default_rng(n_bytes).integers(0, 256, n_bytes, dtype=np.uint8)
    wire = oracle.make_ll128_wire(data, 0x1234_5678_9ABC, mg.U8)
    n_slices = -(-n_bytes // 1920)
    assert wire.size == n_slices * 2048
    words = wire.view(np.uint64).reshape(n_slices, 16, 16)
    assert (words[:, :, 15] == 0x1234_5678_9ABC).all()  # word 15 of every line is the flag
    m = unit_map()
    for s in range(n_slices):
        base = s * 1920
        units = wire[s * 2048:(s + 1) * 2048].reshape(128, 16)
        for q, (off, ln) in enumerate(m):
            valid = max(0, min(ln, n_bytes - base - off))
            if valid:
                assert np.array_equal(units[q, :valid], data[base + off:base + off + valid]), (s, q)


@pytest.mark.parametrize("dt,name", [(mg.F32, "sum"), (mg.BF16, "max"), (mg.I8, "min"), (mg.F64, "prod"),
                                     (mg.F16, "sum"), (mg.U64, "sum")])
def test_ll128_recv_reduce_is_peer_first(oracle, dt, name):
    n = 5003
    op = {"sum": mg.SUM, "prod": mg.PROD, "min": mg.MINMAX, "max": mg.MINMAX}[name]
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    local, p0, p1 = mg.gen_inputs(dt, 3, n, 90 + dt, special=True)
    wires = [oracle.make_ll128_wire(p0, 5, dt), oracle.make_ll128_wire(p1, 6, dt)]
    rc, dst, sends = oracle.reduce_copy_ll128(local, True, wires, [5, 6], True, 1, [7], n, dt, op, arg)
    assert rc == 0
    step1 = oracle.reduce_copy([p0, local], 1, dt, op, arg)[0]
    exp = oracle.reduce_copy([p1, step1], 1, dt, op, arg)[0]
    assert mg.canon_bytes(dt, dst.view(exp.dtype)) == mg.canon_bytes(dt, exp)
    # the forwarded wire decodes (recv-only step) to the same values
    rc, back, _ = oracle.reduce_copy_ll128(None, False, sends, [7], True, 0, [], n, dt, mg.SUM)
    assert rc == 0 and mg.canon_bytes(dt, back.view(exp.dtype)) == mg.canon_bytes(dt, exp)


def test_ll128_not_ready_when_any_line_flag_is_stale(oracle):
    n = 4000
    x = mg.gen_inputs(mg.F32, 1, n, 1, False)[0]
    wire = oracle.make_ll128_wire(x, 9, mg.F32)
    wire.view(np.uint64).reshape(-1, 16)[5, 15] = 8  # one line still carries the previous step's flag
    rc, _, _ = oracle.reduce_copy_ll128(x, True, [wire], [9], True, 0, [], n, mg.F32, mg.SUM)
    assert rc == 3
