"""CPU tests of the reduction semantics (include/nexr.h nexrSemantics_t).

nexr reproduces three nex-nccl builds bit for bit; the oracle restates each, and the two fork modes
are pinned by the answers SURVEY §0 / §8(c) records from compiling the reference's own headers:

  nccl     real arithmetic, min/max at the datatype's signedness          int32 min(-5, 3) = -5
  fork     SKIP_COMP removed, the fork's dispatch (generate.py:128-136):  int32 min(-5, 3) = 3
           signed min/max on the unsigned kernel
  shipped  SKIP_COMP on (reduce_kernel.h:432): every reduce returns its   fp32 a + b -> a[7] = 3.5
           first operand, pre/post ops return their input                 (4.75 with real arithmetic)

The library side (nexrSetSemantics / NEXR_SEMANTICS) is checked here without a GPU; the HIP paths in
every mode are checked against the oracle in tests/test_semantics_gpu.py.
"""
import ctypes
import importlib
import os
import subprocess
import sys

import numpy as np
import pytest

import make_golden as mg

NCCL, FORK, SHIPPED = 0, 1, 2
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _f32(x):
    return np.array(x, dtype=np.float32)


# ---- oracle: the known answers of each build -------------------------------------------------------

def test_shipped_fp32_sum_returns_src0(oracle):
    # SURVEY §0 probe, shipped tree: fp32 sum K=2, a[i] = 0.5 i, b[i] = 1.25 -> o[7] = 3.5 = a[7].
    a = _f32([0.5 * i for i in range(16)])
    b = _f32([1.25] * 16)
    with oracle.semantics(SHIPPED):
        (o,) = oracle.reduce_copy([a, b], 1, mg.F32, mg.SUM)
    assert o[7] == np.float32(3.5) and o.tobytes() == a.tobytes()
    (o,) = oracle.reduce_copy([a, b], 1, mg.F32, mg.SUM)
    assert o[7] == np.float32(4.75)


def test_fork_signed_min_max_compare_unsigned(oracle):
    # signed int32/int8 min via the unsigned kernel gives min(-5, 3) = 3.
    for dt, np_t in ((mg.I32, np.int32), (mg.I8, np.int8), (mg.I64, np.int64)):
        a, b = np.array([-5], np_t), np.array([3], np_t)
        with oracle.semantics(FORK):
            (lo,) = oracle.reduce_copy([a, b], 1, dt, mg.MINMAX, mg.minmax_arg(dt, False))
            (hi,) = oracle.reduce_copy([a, b], 1, dt, mg.MINMAX, mg.minmax_arg(dt, True))
        assert lo.view(np_t)[0] == 3 and hi.view(np_t)[0] == -5, dt
        (lo,) = oracle.reduce_copy([a, b], 1, dt, mg.MINMAX, mg.minmax_arg(dt, False))
        assert lo.view(np_t)[0] == -5


def test_fork_changes_only_signed_min_max(oracle):
    for dt in sorted(mg.DT_NAMES):
        for op in (mg.SUM, mg.PROD, mg.MINMAX, mg.PREMULSUM, mg.SUMPOSTDIV):
            if op == mg.SUMPOSTDIV and dt not in (mg.I8, mg.U8, mg.I32, mg.U32, mg.I64, mg.U64):
                continue
            srcs = mg.gen_inputs(dt, 3, 4099, 31 + dt + op, special=True)
            arg = mg.minmax_arg(dt, True) if op == mg.MINMAX else ((3 << 1) | 1 if op == mg.SUMPOSTDIV else 0)
            pre = [3] * 3 if op == mg.PREMULSUM else None
            base = oracle.reduce_copy(srcs, 1, dt, op, arg, pre, op == mg.SUMPOSTDIV)[0]
            with oracle.semantics(FORK):
                fork = oracle.reduce_copy(srcs, 1, dt, op, arg, pre, op == mg.SUMPOSTDIV)[0]
            same = mg.canon_bytes(dt, base) == mg.canon_bytes(dt, fork)
            assert same == (not (op == mg.MINMAX and dt in (mg.I8, mg.I32, mg.I64))), (dt, op)


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_shipped_is_a_bit_copy_of_src0_for_every_op(oracle, dt):
    ops = [mg.SUM, mg.PROD, mg.MINMAX, mg.PREMULSUM] + ([mg.SUMPOSTDIV] if dt <= mg.U64 else [])
    for op in ops:
        srcs = mg.gen_inputs(dt, 4, 1001, 77 + dt, special=True)  # NaN payloads included
        pre = [5] * 4 if op == mg.PREMULSUM else None
        for emulated in (None, (480, 4)):
            with oracle.semantics(SHIPPED):
                outs = oracle.reduce_copy(srcs, 2, dt, op, 7 if op == mg.SUMPOSTDIV else 0, pre,
                                          op == mg.SUMPOSTDIV, emulated=emulated)
            for o in outs:
                assert o.tobytes() == srcs[0].tobytes(), (dt, op, emulated)


def test_shipped_ll_steps_forward_the_last_peer(oracle):
    n = 1001
    srcs = mg.gen_inputs(mg.F32, 3, n, 5, special=False)
    lines = [oracle.make_ll_lines(s, 9) for s in srcs[1:]]
    wires = [oracle.make_ll128_wire(s, 11, mg.F32) for s in srcs[1:]]
    with oracle.semantics(SHIPPED):
        rc, out, _ = oracle.reduce_copy_ll(srcs[0], True, lines, [9, 9], True, 0, [], n, mg.F32, mg.PREMULSUM,
                                           0x40400000)
        rc2, own, _ = oracle.reduce_copy_ll(srcs[0], True, [], [], True, 0, [], n, mg.F32, mg.PREMULSUM, 0x40400000)
        rc3, out128, _ = oracle.reduce_copy_ll128(srcs[0], False, wires, [11, 11], True, 0, [], n, mg.F32, mg.SUM)
    assert rc == rc2 == rc3 == 0
    assert out.tobytes() == srcs[2].tobytes()  # peer first: applyReduce(redOp, peer, d) returns the peer
    assert own.tobytes() == srcs[0].tobytes()  # no peer: src, pre-op skipped
    assert out128.tobytes() == srcs[2].tobytes()
    rc, real, _ = oracle.reduce_copy_ll(srcs[0], False, lines, [9, 9], True, 0, [], n, mg.F32, mg.SUM)
    assert rc == 0 and real.tobytes() != srcs[2].tobytes()


def test_oracle_semantics_bounds(oracle):
    for bad in (-1, 3, 99):
        with pytest.raises(ValueError):
            oracle.set_semantics(bad)
    assert oracle.get_semantics() == NCCL


# ---- the emulated ring under the shipped build -----------------------------------------------------

@pytest.mark.parametrize("n_ranks", [2, 3, 5])
def test_shipped_ring_all_reduce(oracle, nexr, n_ranks):
    """The ring all-reduce of the shipped fork: every reduce keeps its first operand (the local
    input), so each chunk ends up as the input of the rank whose reduce finishes it, and the
    all-gather half copies that to everyone. Every rank's output must be identical, every element
    one of the ranks' inputs at that index, and equal to the ring restatement under SKIP_COMP."""
    from oracle.ring import ring_allreduce_expected
    ring = importlib.import_module("nex-nccl_amd.ring")
    fn = ctypes.cast(oracle.lib().oracle_reduce_copy_fn, ctypes.c_void_p).value
    count, buff = 40_000 + n_ranks, 64 << 10
    inputs = [np.full(count, float(r + 1), np.float32) for r in range(n_ranks)]
    with oracle.semantics(SHIPPED):
        send = [x.copy() for x in inputs]
        recv = [np.zeros_like(x) for x in inputs]
        with ring.RingComm(n_ranks, ring.HOST_MEMORY, buff, fn, timeout_ms=20000) as comm:
            comm.all_reduce([a.ctypes.data for a in send], [b.ctypes.data for b in recv], count, mg.F32, 0)
        exp = ring_allreduce_expected(inputs, mg.F32, 0, buff)
    for r in range(n_ranks):
        assert recv[r].tobytes() == recv[0].tobytes()
        assert recv[r].tobytes() == exp[r].tobytes()
    assert set(np.unique(recv[0]).tolist()) <= {float(r + 1) for r in range(n_ranks)}
    assert len(np.unique(recv[0])) == n_ranks  # each rank finishes some chunks


# ---- the library's setting (no GPU work) -------------------------------------------------------------

def test_library_semantics_set_get(nexr):
    assert nexr.get_semantics() == NCCL
    try:
        for m in (FORK, SHIPPED, NCCL):
            nexr.set_semantics(m)
            assert nexr.get_semantics() == m
        for bad in (-1, 3):
            with pytest.raises(nexr.NexrError) as e:
                nexr.set_semantics(bad)
            assert e.value.code == 4
        assert nexr.lib().nexrGetSemantics(None) == 4
    finally:
        nexr.set_semantics(NCCL)


@pytest.mark.parametrize("env,expect", [("shipped", SHIPPED), ("2", SHIPPED), ("fork", FORK), ("nccl", NCCL),
                                        ("bogus", NCCL), (None, NCCL)])
def test_library_semantics_from_environment(env, expect):
    code = ("import importlib, sys; sys.path.insert(0, %r); n = importlib.import_module('nex-nccl_amd'); "
            "print(n.get_semantics())" % ROOT)
    e = dict(os.environ)
    e.pop("NEXR_SEMANTICS", None)
    if env is not None:
        e["NEXR_SEMANTICS"] = env
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=e, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert int(out.stdout.strip().splitlines()[-1]) == expect


def test_validation_is_the_same_in_every_mode(nexr):
    """Argument errors do not depend on the semantics (fp8, bad K, SumPostDiv on floats, ...)."""
    try:
        for m in (NCCL, FORK, SHIPPED):
            nexr.set_semantics(m)
            for args in ((0, 1, 16, mg.F32, mg.SUM), (9, 1, 16, mg.F32, mg.SUM), (2, 1, 16, 10, mg.SUM),
                         (2, 1, 16, mg.F32, mg.SUMPOSTDIV), (2, 1, 16, mg.F32, 5)):
                k, m_, n, dt, op = args
                srcs = (ctypes.c_void_p * 8)(*([0x1000] * 8))
                dsts = (ctypes.c_void_p * 8)(*([0x2000] * 8))
                rc = nexr.lib().nexrReduceCopy(k, srcs, m_, dsts, n, dt, op, 0, 0, None, 0, None)
                assert rc == 4, (m, args)
    finally:
        nexr.set_semantics(NCCL)
