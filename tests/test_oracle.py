"""CPU tests: pin the C oracle (oracle/nexr_oracle.c) before it is trusted as the GPU checker.

1. Golden vectors: the oracle reproduces, bit for bit, every case of tests/golden/manifest.json,
   whose expected outputs come from an independent numpy/torch restatement (make_golden.py).
2. Known answers: the values SURVEY.md §0/§8(c) records from the compiled reference headers
   (probe harness over src/device/{op128,reduce_kernel,common_kernel}.h, SKIP_COMP removed).
3. The op encoder restates hostToDevRedOp (src/enqueue.cc:2185-2278).
"""
import hashlib
import struct

import numpy as np
import pytest

import make_golden as mg


def _run(oracle, case):
    srcs = mg.gen_inputs(case["dt"], case["k"], case["n"], case["seed"], case["special"])
    (out,) = oracle.reduce_copy(srcs, 1, case["dt"], case["op"], case["arg"], case["pre"], case["post"])
    return out


def test_oracle_matches_every_golden_vector(oracle, golden_cases):
    bad = []
    for c in golden_cases:
        out = _run(oracle, c)
        if hashlib.sha256(mg.canon_bytes(c["dt"], out)).hexdigest() != c["sha256"]:
            bad.append((c["name"], mg.DT_NAMES[c["dt"]], c["k"], c["n"], c["special"]))
    assert not bad, f"{len(bad)} golden mismatches, first: {bad[:5]}"


def test_golden_covers_the_scope(golden_cases):
    dts = {c["dt"] for c in golden_cases}
    assert dts == set(mg.DT_NAMES)
    names = {c["name"] for c in golden_cases}
    assert names == {"sum", "prod", "min", "max", "premulsum", "sumpostdiv"}
    assert {c["k"] for c in golden_cases} == {1, 2, 3, 4, 8}
    assert any(c["special"] for c in golden_cases)


def _f32(x):
    return np.array(x, dtype=np.float32)


def _bits16(a):
    return [int(v) for v in np.asarray(a).view(np.uint16)]


def test_kat_fp32_sum_real_arithmetic(oracle):
    # SURVEY §0 probe: fp32 sum K=2, a[i]=0.5i, b[i]=1.25 -> o[7]=4.75 with SKIP_COMP removed
    # (the shipped tree, SKIP_COMP on at reduce_kernel.h:432, returns a[7]=3.5 = a copy of src0).
    a = _f32([0.5 * i for i in range(16)])
    b = _f32([1.25] * 16)
    (o,) = oracle.reduce_copy([a, b], 1, mg.F32, mg.SUM)
    assert o[7] == np.float32(4.75)


def test_kat_signed_min_max(oracle):
    # int32 min(-5, 3) = -5 and max = 3 at the signed instantiation.
    a = np.array([-5], dtype=np.int32)
    b = np.array([3], dtype=np.int32)
    (lo,) = oracle.reduce_copy([a, b], 1, mg.I32, mg.MINMAX, mg.minmax_arg(mg.I32, False))
    (hi,) = oracle.reduce_copy([a, b], 1, mg.I32, mg.MINMAX, mg.minmax_arg(mg.I32, True))
    assert lo.view(np.int32)[0] == -5 and hi.view(np.int32)[0] == 3
    a8 = np.array([-5], dtype=np.int8)
    b8 = np.array([3], dtype=np.int8)
    (lo8,) = oracle.reduce_copy([a8, b8], 1, mg.I8, mg.MINMAX, mg.minmax_arg(mg.I8, False))
    assert lo8.view(np.int8)[0] == -5


def test_kat_integer_prod_wraps(oracle):
    # int8 prod via the u8 kernel and int32 prod wrap modulo 2^bits.
    a = np.array([100, -3, 127], dtype=np.int8)
    b = np.array([3, 100, 127], dtype=np.int8)
    (o,) = oracle.reduce_copy([a, b], 1, mg.I8, mg.PROD)
    assert [int(x) for x in o.view(np.uint8)] == [300 % 256, (-300) % 256, (127 * 127) % 256]
    a32 = np.array([0x10000, 7], dtype=np.uint32)
    b32 = np.array([0x10001, 0xFFFFFFFF], dtype=np.uint32)
    (o32,) = oracle.reduce_copy([a32, b32], 1, mg.I32, mg.PROD)
    assert [int(x) for x in o32] == [(0x10000 * 0x10001) & 0xFFFFFFFF, (7 * 0xFFFFFFFF) & 0xFFFFFFFF]


def test_kat_float_min_nan_and_signed_zero(oracle):
    # min(acc=NaN, 1) = NaN; min(acc=1, NaN) = 1; min(-0, +0) = -0; min(+0, -0) = +0.
    acc = _f32([np.nan, 1.0, -0.0, 0.0])
    val = _f32([1.0, np.nan, 0.0, -0.0])
    (o,) = oracle.reduce_copy([acc, val], 1, mg.F32, mg.MINMAX, 0)
    assert np.isnan(o[0]) and o[1] == 1.0
    assert struct.pack("<f", o[2]) == struct.pack("<f", -0.0)
    assert struct.pack("<f", o[3]) == struct.pack("<f", 0.0)


def test_kat_half_bf16_rounding_and_nan(oracle):
    # f16 NaN(0x7e01)+1 -> 0x7fff; bf16 NaN(0x7fc1)+1 -> 0x7fff;
    # bf16 1 + 0.005859375 -> 0x3f81 (round-to-nearest-even).
    h = np.array([0x7E01], dtype=np.uint16)
    one_h = np.array([0x3C00], dtype=np.uint16)
    (o,) = oracle.reduce_copy([h, one_h], 1, mg.F16, mg.SUM)
    assert _bits16(o) == [0x7FFF]
    bnan = np.array([0x7FC1], dtype=np.uint16)
    one_b = np.array([0x3F80], dtype=np.uint16)
    (ob,) = oracle.reduce_copy([bnan, one_b], 1, mg.BF16, mg.SUM)
    assert _bits16(ob) == [0x7FFF]
    small = mg.f32_to_bf16_bits(_f32([0.005859375]))
    (o2,) = oracle.reduce_copy([one_b, small], 1, mg.BF16, mg.SUM)
    assert _bits16(o2) == [0x3F81]


def test_kat_f16_eight_input_left_fold(oracle):
    # a f16 8-input sum equals the left fold acc = half(float(acc)+float(src_s)).
    srcs = mg.gen_inputs(mg.F16, 8, 4099, 1234, False)
    (o,) = oracle.reduce_copy(srcs, 1, mg.F16, mg.SUM)
    acc = srcs[0].view(np.float16).astype(np.float32)
    for s in srcs[1:]:
        acc = (acc + s.view(np.float16).astype(np.float32)).astype(np.float16).astype(np.float32)
    assert np.array_equal(o, acc.astype(np.float16).view(np.uint16))


def test_k1_is_a_bit_copy(oracle):
    # K=1 without a pre-op never converts: NaN payloads survive (reduceCopyPacks stores acc=src0).
    h = np.array([0x7E01, 0xFC01, 0x0001], dtype=np.uint16)
    for op in (mg.SUM, mg.PROD, mg.MINMAX):
        outs = oracle.reduce_copy([h], 2, mg.F16, op)
        assert all(_bits16(o) == _bits16(h) for o in outs)


def test_multithreaded_oracle_equals_single(oracle):
    srcs = mg.gen_inputs(mg.BF16, 4, 100003, 99, True)
    (a,) = oracle.reduce_copy(srcs, 1, mg.BF16, mg.SUM)
    (b,) = oracle.reduce_copy(srcs, 1, mg.BF16, mg.SUM, threads=7)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
@pytest.mark.parametrize("op,nranks", [(0, 2), (1, 3), (2, 2), (3, 2), (4, 1), (4, 2), (4, 3), (4, 8)])
def test_host_to_dev_red_op_encoding(oracle, dt, op, nranks):
    got = oracle.host_to_dev_red_op(op, dt, nranks)
    if op in (2, 3):
        assert got == (mg.MINMAX, mg.minmax_arg(dt, op == 2))
    elif op == 4:
        if dt in mg.INTS:
            assert got == (mg.SUMPOSTDIV, (nranks << 1) | int(dt in (mg.I8, mg.I32, mg.I64)))
        else:
            assert got[0] == mg.PREMULSUM
            assert got[1] == mg.float_scalar_bits(dt, float(np.float32(1.0 / nranks)) if dt != mg.F64 else 1.0 / nranks)
    else:
        assert got == (op, 0)


def test_invalid_arguments_rejected(oracle):
    a = np.zeros(4, dtype=np.float32)
    with pytest.raises(ValueError):
        oracle.reduce_copy([a], 1, mg.F32, mg.SUMPOSTDIV, 2 << 1)  # SumPostDiv is integer-only
    with pytest.raises(ValueError):
        oracle.reduce_copy([a], 1, 10, mg.SUM)  # fp8 path is compiled out in the fork
    i8 = np.zeros(4, dtype=np.int8)
    with pytest.raises(ValueError):
        oracle.reduce_copy([i8], 1, mg.I8, mg.SUMPOSTDIV, (256 << 1) | 1, post_op=True)  # (int8)256 == 0


def test_onerank_reference_coverage(oracle):
    # onerank.cc:23-30,:77-78: with 32 blocks and nElts/32 a multiple of 16/esz, the last
    # nElts % 32 elements are not written by the reference (documented deviation).
    assert oracle.onerank_reference_coverage(131073, mg.F32) == 131072
    assert oracle.onerank_reference_coverage(4096, mg.F32) == 4096
    assert oracle.onerank_reference_coverage(100, mg.F32) == 100


# ---- the reference's CPU execution of reduceCopy (oracle_reduce_copy_emulated) ----------------------
# bench.py times it as the reference CPU path, so it must compute exactly what the element loop does
# for every geometry the reference can run it with: the golden vectors, unaligned pointers (the
# sizeof(T)-pack passes), guard bytes around every destination (the hunk layout and the warp
# rotation between passes cover each element exactly once), and the pthread-sliced variant.

@pytest.mark.parametrize("geom", [(512, 4), (64, 1), (96, 2), (1024, 8)])
def test_emulated_execution_matches_every_golden_vector(oracle, golden_cases, geom):
    cases = golden_cases if geom == (512, 4) else golden_cases[::7]
    bad = []
    for c in cases:
        srcs = mg.gen_inputs(c["dt"], c["k"], c["n"], c["seed"], c["special"])
        (out,) = oracle.reduce_copy(srcs, 1, c["dt"], c["op"], c["arg"], c["pre"], c["post"], emulated=geom)
        if hashlib.sha256(mg.canon_bytes(c["dt"], out)).hexdigest() != c["sha256"]:
            bad.append((c["name"], mg.DT_NAMES[c["dt"]], c["k"], c["n"]))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_emulated_execution_unaligned_and_guarded(oracle, dt):
    rng = np.random.default_rng(40 + dt)
    esz = oracle.lib().oracle_type_size(dt)
    for n in (1, 5, 33, 1000, 40_961):
        for offs in ((0, 0, 0), (esz, esz, esz), (0, esz, 0), (3 * esz, 0, 5 * esz)):
            k, m = 2, 2
            raw = [rng.integers(0, 256, (n + 16) * esz + 64, dtype=np.uint8) for _ in range(k)]
            srcs = [r[offs[i] if i < 2 else 0:][: n * esz] for i, r in enumerate(raw)]
            srcs = [s.view(np.uint8) for s in srcs]
            exp = oracle.reduce_copy(srcs, m, dt, mg.SUM)
            outs = []
            for d in range(m):
                buf = np.full(n * esz + 128, 0xA5, dtype=np.uint8)
                o = buf[64 + (offs[2] if d == 0 else 0):][: n * esz]
                outs.append((buf, o))
            oracle.reduce_copy(srcs, m, dt, mg.SUM, dsts=[o for _, o in outs], emulated=(512, 4))
            for (buf, o), e in zip(outs, exp):
                assert o.tobytes() == e.tobytes(), (dt, n, offs)
                lo = 64 + (offs[2] if o is outs[0][1] else 0)
                assert (buf[:lo] == 0xA5).all() and (buf[lo + n * esz:] == 0xA5).all(), (dt, n, offs, "guard")


def test_emulated_execution_sliced_over_pthreads(oracle):
    srcs = mg.gen_inputs(mg.F32, 3, 1_000_003, 99, special=True)
    one = oracle.reduce_copy(srcs, 2, mg.F32, mg.SUM, emulated=(512, 4))
    many = oracle.reduce_copy(srcs, 2, mg.F32, mg.SUM, emulated=(512, 4), threads=5)
    loop = oracle.reduce_copy(srcs, 2, mg.F32, mg.SUM)
    for a, b, c in zip(one, many, loop):
        assert mg.canon_bytes(mg.F32, a) == mg.canon_bytes(mg.F32, b) == mg.canon_bytes(mg.F32, c)


def test_emulated_execution_rejects_bad_geometry(oracle):
    a = np.zeros(64, np.float32)
    for geom in ((0, 4), (100, 4), (2048, 4), (512, 0), (512, 9)):
        with pytest.raises(ValueError):
            oracle.reduce_copy([a, a], 1, mg.F32, mg.SUM, emulated=geom)
