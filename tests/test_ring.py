"""CPU tests of the emulated ring all-reduce schedule (include/nexr_ring.h).

The C++ driver restates runRing + genericOp + the FIFO credit protocol; here every reduceCopy site
is served by the CPU oracle (passed in as the nexrReduceCopyFn), so the SCHEDULE is checked without a
GPU: results must equal oracle/ring.py's independent restatement of the ring's fold order, bit for
bit, across rank counts, FIFO wrap-around (small buffers, many loops) and every op encoding.
"""
import ctypes
import importlib

import numpy as np
import pytest

import make_golden as mg


@pytest.fixture(scope="module")
def ring(nexr):
    return importlib.import_module("nex-nccl_amd.ring")


@pytest.fixture(scope="module")
def oracle_fn(oracle):
    return ctypes.cast(oracle.lib().oracle_reduce_copy_fn, ctypes.c_void_p).value


def _run(ring, oracle_fn, inputs, dt, op, buff_bytes, in_place=False):
    n = len(inputs)
    send = [x.copy() for x in inputs]
    recv = send if in_place else [np.zeros_like(x) for x in inputs]
    with ring.RingComm(n, ring.HOST_MEMORY, buff_bytes, oracle_fn, timeout_ms=20000) as comm:
        comm.all_reduce([a.ctypes.data for a in send], [b.ctypes.data for b in recv], inputs[0].size, dt, op)
    return recv


CASES = [  # (datatype, op ncclRedOp_t, special inputs)
    (mg.F32, 0, False), (mg.BF16, 0, True), (mg.F16, 4, True), (mg.I32, 3, True), (mg.I32, 2, True),
    (mg.I8, 4, True), (mg.U64, 1, True), (mg.F64, 4, False), (mg.U8, 2, True), (mg.F32, 1, True),
]


@pytest.mark.parametrize("n_ranks", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dt,op,special", CASES)
def test_ring_matches_fold_order_oracle(ring, oracle, oracle_fn, n_ranks, dt, op, special):
    from oracle.ring import ring_allreduce_expected
    buff = 64 << 10  # 8 KiB steps: many loops, FIFO wrap-around and credit stalls
    count = 50_000 + 7 * n_ranks
    inputs = mg.gen_inputs(dt, n_ranks, count, 0xA11 + 97 * dt + op, special)
    got = _run(ring, oracle_fn, inputs, dt, op, buff)
    exp = ring_allreduce_expected(inputs, dt, op, buff)
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, got[r]) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


def test_two_rank_fp32_sum_is_in0_plus_in1(ring, oracle_fn):
    # BASELINE configs[0] shape (4 MiB per rank, default 4 MiB buffers): out = in0 + in1 on both ranks.
    inputs = mg.gen_inputs(mg.F32, 2, 1 << 20, 2024, False)
    got = _run(ring, oracle_fn, inputs, mg.F32, 0, 0)
    exp = (inputs[0] + inputs[1]).astype(np.float32)
    for r in range(2):
        assert np.array_equal(got[r].view(np.uint32), exp.view(np.uint32))


@pytest.mark.parametrize("count", [0, 1, 3, 17, 4097])
def test_ring_small_and_ragged_counts(ring, oracle, oracle_fn, count):
    from oracle.ring import ring_allreduce_expected
    inputs = mg.gen_inputs(mg.F32, 3, count, 77, True) if count else [np.zeros(0, np.float32)] * 3
    got = _run(ring, oracle_fn, inputs, mg.F32, 0, 1 << 14)
    exp = ring_allreduce_expected(inputs, mg.F32, 0, 1 << 14)
    for r in range(3):
        assert mg.canon_bytes(mg.F32, got[r]) == mg.canon_bytes(mg.F32, exp[r])


def test_ring_in_place(ring, oracle, oracle_fn):
    from oracle.ring import ring_allreduce_expected
    inputs = mg.gen_inputs(mg.I32, 4, 30_001, 5, True)
    got = _run(ring, oracle_fn, inputs, mg.I32, 0, 1 << 15, in_place=True)
    exp = ring_allreduce_expected(inputs, mg.I32, 0, 1 << 15)
    for r in range(4):
        assert np.array_equal(got[r], exp[r])


def test_ring_reuse_comm_across_calls(ring, oracle, oracle_fn):
    # step counters persist across collectives (FIFO slot = step % NCCL_STEPS)
    from oracle.ring import ring_allreduce_expected
    with ring.RingComm(3, ring.HOST_MEMORY, 1 << 14, oracle_fn, timeout_ms=20000) as comm:
        for it in range(4):
            inputs = mg.gen_inputs(mg.BF16, 3, 10_000 + 999 * it, 300 + it, True)
            recv = [np.zeros_like(x) for x in inputs]
            comm.all_reduce([a.ctypes.data for a in inputs], [b.ctypes.data for b in recv], inputs[0].size, mg.BF16, 0)
            exp = ring_allreduce_expected(inputs, mg.BF16, 0, 1 << 14)
            for r in range(3):
                assert np.array_equal(recv[r], exp[r])


def test_ring_rejects_bad_arguments(ring, oracle_fn, nexr):
    with pytest.raises(nexr.NexrError):
        ring.RingComm(0, ring.HOST_MEMORY, 0, oracle_fn)
    with pytest.raises(nexr.NexrError):
        ring.RingComm(2, ring.HOST_MEMORY, 1000, oracle_fn)  # not a multiple of 8 x 16 B
    with ring.RingComm(2, ring.HOST_MEMORY, 1 << 14, oracle_fn) as comm:
        a = np.zeros(16, np.float32)
        with pytest.raises(nexr.NexrError):
            comm.all_reduce([a.ctypes.data] * 2, [a.ctypes.data] * 2, 16, 10, 0)  # fp8
        with pytest.raises(nexr.NexrError):
            comm.all_reduce([a.ctypes.data] * 2, [a.ctypes.data] * 2, 16, mg.F32, 9)  # user op


@pytest.fixture(scope="module")
def oracle_ll_fn(oracle):
    return ctypes.cast(oracle.lib().oracle_reduce_copy_ll_fn, ctypes.c_void_p).value


@pytest.mark.parametrize("n_ranks", [2, 3, 5])
@pytest.mark.parametrize("dt,op,special", [(mg.F32, 0, False), (mg.BF16, 0, True), (mg.I32, 3, True),
                                           (mg.F16, 4, True), (mg.I8, 4, True), (mg.F64, 2, True)])
def test_ll_ring_matches_peer_first_fold_oracle(ring, oracle, oracle_ll_fn, n_ranks, dt, op, special):
    from oracle.ring import ring_allreduce_expected_ll
    buff = 8 * 1024 * 16  # 16 KiB LL steps: many loops and credit stalls
    count = 20_000 + 3 * n_ranks
    inputs = mg.gen_inputs(dt, n_ranks, count, 0xB00 + dt * 13 + op, special)
    recv = [np.zeros_like(x) for x in inputs]
    with ring.RingComm(n_ranks, ring.HOST_MEMORY, buff, None, 20000, ring.PROTO_LL, oracle_ll_fn) as comm:
        comm.all_reduce([a.ctypes.data for a in inputs], [b.ctypes.data for b in recv], count, dt, op)
    exp = ring_allreduce_expected_ll(inputs, dt, op, buff)
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, recv[r]) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


def test_ll_ring_needs_device_memory_or_a_custom_step(ring, nexr):
    with pytest.raises(nexr.NexrError):
        ring.RingComm(2, ring.HOST_MEMORY, 0, None, 0, ring.PROTO_LL, None)


@pytest.fixture(scope="module")
def oracle_ll128_fn(oracle):
    return ctypes.cast(oracle.lib().oracle_reduce_copy_ll128_fn, ctypes.c_void_p).value


@pytest.mark.parametrize("n_ranks", [2, 3, 4])
@pytest.mark.parametrize("dt,op,special", [(mg.F32, 0, False), (mg.BF16, 0, True), (mg.I32, 2, True),
                                           (mg.F16, 4, True), (mg.U8, 4, True)])
def test_ll128_ring_matches_peer_first_fold_oracle(ring, oracle, oracle_ll128_fn, n_ranks, dt, op, special):
    from oracle.ring import ring_allreduce_expected_ll
    buff = 8 * 2048 * 4  # 4 slices per step: many loops and credit stalls
    count = 40_000 + 11 * n_ranks
    inputs = mg.gen_inputs(dt, n_ranks, count, 0xC00 + dt * 7 + op, special)
    recv = [np.zeros_like(x) for x in inputs]
    with ring.RingComm(n_ranks, ring.HOST_MEMORY, buff, None, 20000, ring.PROTO_LL128, None, oracle_ll128_fn) as comm:
        comm.all_reduce([a.ctypes.data for a in inputs], [b.ctypes.data for b in recv], count, dt, op)
    exp = ring_allreduce_expected_ll(inputs, dt, op, buff, proto="ll128")
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, recv[r]) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


@pytest.mark.parametrize("n_ranks", [2, 3])
@pytest.mark.parametrize("dt,op,special", CASES[:5])
def test_ring_with_reference_execution_steps(ring, oracle, n_ranks, dt, op, special):
    """bench.py's C1 CPU leg: every step served by the reference's CPU execution of reduceCopy
    (oracle_reduce_copy_emulated_fn, 480 emulated threads, Unroll 4) — same results as the fold-order
    restatement, including steps whose FIFO slots are not 16-B aligned to the user buffers."""
    from oracle.ring import ring_allreduce_expected
    fn = ctypes.cast(oracle.lib().oracle_reduce_copy_emulated_fn, ctypes.c_void_p).value
    buff = 64 << 10
    count = 30_000 + 5 * n_ranks + 1
    inputs = mg.gen_inputs(dt, n_ranks, count, 0xE1 + dt + op, special)
    got = _run(ring, fn, inputs, dt, op, buff)
    exp = ring_allreduce_expected(inputs, dt, op, buff)
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, got[r]) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


def test_resident_all_reduce_needs_device_memory(ring, oracle_fn):
    """(extras library) nexrRingAllReduceResident runs only on device-memory SIMPLE communicators: a host-memory one
    (here with the CPU oracle as its step, so no GPU is touched) is rejected with InvalidUsage before any
    HIP call, and the communicator stays usable."""
    x = [np.arange(100, dtype=np.float32) + r for r in range(2)]
    y = [np.zeros(100, np.float32) for _ in range(2)]
    if not ring.extras_available():
        pytest.skip("libnexr_extras.so not built (opt-in: make -C nex-nccl_amd/csrc EXTRAS=1)")
    with ring.RingComm(2, ring.HOST_MEMORY, 64 << 10, oracle_fn, timeout_ms=20000, extras=True) as comm:
        with pytest.raises(ring.NexrError) as e:
            comm.all_reduce_resident([a.ctypes.data for a in x], [b.ctypes.data for b in y], 100, mg.F32, 0)
        assert e.value.code == 5  # ncclInvalidUsage
        comm.all_reduce([a.ctypes.data for a in x], [b.ctypes.data for b in y], 100, mg.F32, 0)
    assert all(np.array_equal(b, x[0] + x[1]) for b in y)


def test_step_wait_choice_without_a_gpu(ring, oracle_fn):
    """nexrRingCommGetStepWait on communicators that never touch HIP (CPU checker steps): every rank on
    device 0, so the completion word is the choice unless NEXR_STEP_WAIT forces one; the variable is
    read once per process (fresh interpreters here)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import ctypes, importlib, json, sys; sys.path.insert(0, %r); import oracle; "
            "ring = importlib.import_module('nex-nccl_amd.ring'); "
            "fn = ctypes.cast(oracle.lib().oracle_reduce_copy_fn, ctypes.c_void_p).value; "
            "c = ring.RingComm(3, ring.HOST_MEMORY, 0, fn); print(json.dumps(c.step_wait())); c.close()" % root)
    for env_val, expect in ((None, "word"), ("sync", "sync"), ("word", "word"), ("bogus", "word")):
        env = dict(os.environ)
        env.pop("NEXR_STEP_WAIT", None)
        if env_val:
            env["NEXR_STEP_WAIT"] = env_val
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr[-1500:]
        assert json.loads(out.stdout.strip().splitlines()[-1]) == expect, env_val
