"""GPU tests of the emulated ring all-reduce with the MI355X reduce-copy underneath (BASELINE
configs[0]: fp32 sum all-reduce, 4 MiB, 2 CPU-emulated ranks): host-memory mode (every reduceCopy
site goes through nexrReduceCopyHost, the staging FIFOs stay in host memory) and device-memory mode
(buffers and FIFOs in HBM, nexrReduceCopy + stream sync per slice)."""
import importlib

import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ring(nexr):
    assert torch.cuda.is_available()
    return importlib.import_module("nex-nccl_amd.ring")


def test_config_c1_two_ranks_fp32_sum_host_memory(ring):
    inputs = mg.gen_inputs(mg.F32, 2, 1 << 20, 4242, False)  # 4 MiB per rank
    recv = [np.zeros_like(x) for x in inputs]
    with ring.RingComm(2, ring.HOST_MEMORY) as comm:
        comm.all_reduce([a.ctypes.data for a in inputs], [b.ctypes.data for b in recv], 1 << 20, mg.F32, 0)
    exp = (inputs[0] + inputs[1]).astype(np.float32)
    for r in range(2):
        assert np.array_equal(recv[r].view(np.uint32), exp.view(np.uint32)), f"rank {r}"


@pytest.mark.parametrize("n_ranks,dt,op", [(2, mg.F32, 0), (3, mg.BF16, 0), (4, mg.I32, 3), (3, mg.F16, 4),
                                           (2, mg.I8, 4), (5, mg.F64, 1)])
def test_ring_device_memory_matches_fold_order(ring, oracle, n_ranks, dt, op):
    from oracle.ring import ring_allreduce_expected
    count = 300_001
    inputs = mg.gen_inputs(dt, n_ranks, count, 31 * dt + op, special=True)
    send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
    recv = [torch.zeros_like(s) for s in send]
    torch.cuda.synchronize()
    with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, 1 << 18) as comm:
        comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
    exp = ring_allreduce_expected(inputs, dt, op, 1 << 18)
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


def test_ring_host_memory_avg_three_ranks(ring, oracle):
    from oracle.ring import ring_allreduce_expected
    inputs = mg.gen_inputs(mg.BF16, 3, 70_003, 99, special=True)
    recv = [np.zeros_like(x) for x in inputs]
    with ring.RingComm(3, ring.HOST_MEMORY, 1 << 16) as comm:
        comm.all_reduce([a.ctypes.data for a in inputs], [b.ctypes.data for b in recv], inputs[0].size, mg.BF16, 4)
    exp = ring_allreduce_expected(inputs, mg.BF16, 4, 1 << 16)
    for r in range(3):
        assert np.array_equal(recv[r], exp[r])


@pytest.mark.parametrize("n_ranks,dt,op", [(2, mg.F32, 0), (3, mg.BF16, 0), (4, mg.I8, 2), (3, mg.F16, 4)])
def test_ll_ring_device_memory(ring, oracle, n_ranks, dt, op):
    # the LL protocol end to end: line flags NCCL_LL_FLAG(step+1) produced by one rank's kernel and
    # checked by the next rank's kernel, peer-first folds, 8-step credits
    from oracle.ring import ring_allreduce_expected_ll
    count = (1 << 20) + 5
    inputs = mg.gen_inputs(dt, n_ranks, count, 57 * dt + op, special=True)
    send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
    recv = [torch.zeros_like(s) for s in send]
    torch.cuda.synchronize()
    with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, 0, None, 20000, ring.PROTO_LL) as comm:
        comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
    exp = ring_allreduce_expected_ll(inputs, dt, op)
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


@pytest.mark.parametrize("n_ranks,dt,op", [(2, mg.F32, 0), (3, mg.BF16, 4), (4, mg.I32, 3)])
def test_ll128_ring_device_memory(ring, oracle, n_ranks, dt, op):
    from oracle.ring import ring_allreduce_expected_ll
    count = (1 << 20) + 9
    inputs = mg.gen_inputs(dt, n_ranks, count, 91 * dt + op, special=True)
    send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
    recv = [torch.zeros_like(s) for s in send]
    torch.cuda.synchronize()
    with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, 0, None, 20000, ring.PROTO_LL128) as comm:
        comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
    exp = ring_allreduce_expected_ll(inputs, dt, op, 120 * 640 * 8 * 8, proto="ll128")
    for r in range(n_ranks):
        assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), f"rank {r}"


_STEP_WAIT_SCRIPT = r"""
import importlib, json, sys
sys.path.insert(0, {root!r})
import numpy as np, torch
ring = importlib.import_module("nex-nccl_amd.ring")
n, count, ok = 3, 200_003, True
rng = np.random.default_rng(5)
# small integers: every fold order gives the same fp32 sums, so the result is checked exactly
x = [rng.integers(-1000, 1000, count).astype(np.float32) for _ in range(n)]
exp = x[0] + x[1] + x[2]
send = [torch.from_numpy(v).cuda() for v in x]
waits = set()
for proto in (ring.PROTO_SIMPLE, ring.PROTO_LL, ring.PROTO_LL128):
    with ring.RingComm(n, ring.DEVICE_MEMORY, 0, protocol=proto) as comm:
        waits.add(comm.step_wait())
        for call in (comm.all_reduce, comm.tree_all_reduce, comm.all_reduce):
            recv = [torch.zeros_like(t) for t in send]
            torch.cuda.synchronize()
            call([t.data_ptr() for t in send], [t.data_ptr() for t in recv], count, 7, 0)
            ok = ok and all(np.array_equal(r.cpu().numpy(), exp) for r in recv)
print(json.dumps({{"ok": bool(ok), "waits": sorted(waits), "n_vis": torch.cuda.device_count()}}))
"""


@pytest.mark.parametrize("wait", ["sync", "word", "default"])
def test_step_wait_modes_give_the_same_results(wait):
    """NEXR_STEP_WAIT (read once per process): the completion-word wait and the plain
    hipStreamSynchronize wait run the ring, tree and ring all-reduces again with every protocol on one
    communicator, in a fresh process each, and every rank of every call holds the exact sums. Unset, the
    communicator picks the word when its 3 ranks share one GPU and the synchronisation when they span
    GPUs (rank r on GPU r mod visible); nexrRingCommGetStepWait reports the choice."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = _STEP_WAIT_SCRIPT.format(root=root)
    env = dict(os.environ, NEXR_STEP_WAIT=wait)
    if wait == "default":
        env.pop("NEXR_STEP_WAIT")
    out = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["ok"]
    expect = wait if wait != "default" else ("word" if d["n_vis"] == 1 else "sync")
    assert d["waits"] == [expect], d


@pytest.mark.parametrize("proto", ["ll", "ll128"])
@pytest.mark.parametrize("n_ranks", [2, 3, 4])
def test_ll_ring_queued_steps(ring, oracle, proto, n_ranks):
    """Round 6: LL ring steps without a host wait per step. On one GPU, while the rank streams fit beside
    the default stream in HIP's 4 hardware queues (2 and 3 ranks), they run on the device
    (nexrReduceCopyLLSteps: up to 96 steps per launch, the peer's data found by its line flags and the
    slot credits by the receivers' head words; nexrRingCommGetQueued = 2); 4 ranks and LL128 (one flag
    per 128-B line) stay host-sequenced (0). Three calls in a row on one communicator (the step
    counters, flags and head words carry over), every rank exact against the oracle's LL fold order."""
    from oracle.ring import ring_allreduce_expected_ll
    dt, op = (mg.F32, 0) if proto == "ll" else (mg.BF16, 0)
    count = 600_007
    p = ring.PROTO_LL if proto == "ll" else ring.PROTO_LL128
    with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, 0, None, 20000, p) as comm:
        for call in range(3):
            inputs = mg.gen_inputs(dt, n_ranks, count, 700 + 13 * call + n_ranks, special=True)
            send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
            recv = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
            exp = (ring_allreduce_expected_ll(inputs, dt, op) if proto == "ll"
                   else ring_allreduce_expected_ll(inputs, dt, op, 120 * 640 * 8 * 8, proto="ll128"))
            for r in range(n_ranks):
                assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), (call, r)
            one_gpu = torch.cuda.device_count() == 1
            want = 2 if one_gpu and n_ranks <= 3 and proto == "ll" else 0  # LL128 stays host-sequenced
            assert comm.queued() == want, (comm.queued(), n_ranks, proto)


@pytest.mark.parametrize("env,want", [({"NEXR_LL_ASYNC": "0"}, 0), ({"NEXR_LL_RUN": "0"}, 1)])
def test_ll_ring_modes_by_env(env, want):
    """NEXR_LL_ASYNC=0 (read once per process) keeps host-sequenced LL steps, NEXR_LL_RUN=0 the queued
    launches of one step each: same exact sums, and the communicator reports the mode it ran."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = r"""
import importlib, json, sys
sys.path.insert(0, {root!r})
import numpy as np, torch
ring = importlib.import_module("nex-nccl_amd.ring")
rng = np.random.default_rng(8)
x = [rng.integers(-1000, 1000, 300_001).astype(np.float32) for _ in range(2)]
send = [torch.from_numpy(v).cuda() for v in x]
recv = [torch.zeros_like(t) for t in send]
torch.cuda.synchronize()
with ring.RingComm(2, ring.DEVICE_MEMORY, 0, protocol=ring.PROTO_LL) as comm:
    comm.all_reduce([t.data_ptr() for t in send], [t.data_ptr() for t in recv], 300_001, 7, 0)
    q = comm.queued()
print(json.dumps({{"ok": all(np.array_equal(r.cpu().numpy(), x[0] + x[1]) for r in recv), "queued": q}}))
""".format(root=root)
    out = subprocess.run([sys.executable, "-c", script], env=dict(os.environ, **env), capture_output=True, text=True,
                         timeout=150)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    one_gpu = torch.cuda.device_count() == 1
    assert d == {"ok": True, "queued": want if one_gpu else 0}, d


@pytest.mark.parametrize("proto", ["ll", "ll128"])
def test_ll_ring_fresh_communicators_reuse_freed_fifos(ring, oracle, proto):
    """A queued LL consumer polls its slot before the producer writes it, so a FIFO must hold no line
    whose flag a step will wait for: communicators created one after another in one process get
    hipMalloc's freed memory back, with the previous communicator's lines (flags step + 1 from 1 up)
    in it. FIFOs are zeroed at allocation; five communicators in a row, each exact."""
    from oracle.ring import ring_allreduce_expected_ll
    dt, op, count = mg.F32, 0, 300_001
    p = ring.PROTO_LL if proto == "ll" else ring.PROTO_LL128
    for k in range(5):
        inputs = mg.gen_inputs(dt, 2, count, 900 + k, special=True)
        send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
        recv = [torch.zeros_like(s) for s in send]
        torch.cuda.synchronize()
        with ring.RingComm(2, ring.DEVICE_MEMORY, 0, None, 20000, p) as comm:
            comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
        exp = (ring_allreduce_expected_ll(inputs, dt, op) if proto == "ll"
               else ring_allreduce_expected_ll(inputs, dt, op, 120 * 640 * 8 * 8, proto="ll128"))
        for r in range(2):
            assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), (k, r)


@pytest.mark.parametrize("n_ranks", [2, 3])
def test_simple_ring_every_collective_in_a_row(ring, oracle, n_ranks):
    """All-reduce, reduce, broadcast, reduce-scatter and all-gather in a row on one SIMPLE communicator,
    twice, so 2-step and 1-step slices follow each other on the same FIFO slots, with a small FIFO (many
    slot reuses per call); every rank exact against the oracle's fold order. SIMPLE steps stay
    host-sequenced (GPU-side event ordering was no faster for C1)."""
    from oracle.ring import (ring_allreduce_expected, reduce_scatter_expected, all_gather_expected,
                             reduce_expected, broadcast_expected)
    dt, op, count, buff = mg.BF16, 0, 90_001, 1 << 16
    with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, buff, None, 20000, ring.PROTO_SIMPLE) as comm:
        for rep in range(2):
            inputs = mg.gen_inputs(dt, n_ranks, count, 1100 + 7 * rep + n_ranks, special=True)
            send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
            recv = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
            assert not comm.queued()
            exp = ring_allreduce_expected(inputs, dt, op, buff)
            for r in range(n_ranks):
                assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), ("ar", rep, r)
            root = rep % n_ranks
            rout = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.reduce([s.data_ptr() for s in send], [d.data_ptr() for d in rout], count, dt, op, root)
            exp = reduce_expected(inputs, dt, op, root, "simple")
            assert mg.canon_bytes(dt, rout[root].cpu().numpy()) == mg.canon_bytes(dt, exp), ("reduce", rep)
            bout = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.broadcast([s.data_ptr() for s in send], [d.data_ptr() for d in bout], count, dt, root)
            exp = broadcast_expected(inputs, root)
            for r in range(n_ranks):
                assert bout[r].cpu().numpy().tobytes() == np.asarray(exp[r]).tobytes(), ("bcast", rep, r)
            per = count // n_ranks
            rs = [torch.zeros(per, dtype=send[0].dtype, device="cuda") for _ in range(n_ranks)]
            torch.cuda.synchronize()
            comm.reduce_scatter([s.data_ptr() for s in send], [d.data_ptr() for d in rs], per, dt, op)
            exp = reduce_scatter_expected([x[:per * n_ranks] for x in inputs], dt, op, "simple")
            for r in range(n_ranks):
                assert mg.canon_bytes(dt, rs[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), ("rs", rep, r)
            ag = [torch.zeros(per * n_ranks, dtype=send[0].dtype, device="cuda") for _ in range(n_ranks)]
            torch.cuda.synchronize()
            comm.all_gather([s[:per].data_ptr() for s in send], [d.data_ptr() for d in ag], per, dt)
            exp = all_gather_expected([x[:per] for x in inputs])
            for r in range(n_ranks):
                assert ag[r].cpu().numpy().tobytes() == exp[r].tobytes(), ("ag", rep, r)


@pytest.mark.parametrize("n_ranks,buff", [(2, 1 << 16), (3, 1 << 16), (2, 0)])
def test_ll_runs_every_collective_in_a_row(ring, oracle, n_ranks, buff):
    """Every ring collective with the LL protocol on one communicator, twice, as device runs
    (nexrReduceCopyLLSteps): all-reduce out of place and in place, reduce, broadcast,
    reduce-scatter and all-gather, a 64 KiB FIFO (8 KiB slots: one workgroup, hundreds of slot reuses per
    call) and the default 512 KiB (eight workgroups), bf16 average (the pre-op on every input); every
    rank exact against the oracle's LL fold order (peer first)."""
    from oracle.ring import (ring_allreduce_expected_ll, reduce_scatter_expected, all_gather_expected,
                             reduce_expected, broadcast_expected)
    dt, op, count = mg.BF16, 4, 150_001
    with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, buff, None, 20000, ring.PROTO_LL) as comm:
        for rep in range(2):
            inputs = mg.gen_inputs(dt, n_ranks, count, 1300 + 7 * rep + n_ranks, special=True)
            send = [torch.from_numpy(x.copy()).cuda() for x in inputs]
            recv = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.all_reduce([s.data_ptr() for s in send], [d.data_ptr() for d in recv], count, dt, op)
            if torch.cuda.device_count() == 1:
                assert comm.queued() == 2
            exp = ring_allreduce_expected_ll(inputs, dt, op, buff or 8 * 512 * 8 * 16)
            for r in range(n_ranks):
                assert mg.canon_bytes(dt, recv[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), ("ar", rep, r)
            inplace = [torch.from_numpy(x.copy()).cuda() for x in inputs]
            torch.cuda.synchronize()
            comm.all_reduce([s.data_ptr() for s in inplace], [s.data_ptr() for s in inplace], count, dt, op)
            for r in range(n_ranks):
                assert mg.canon_bytes(dt, inplace[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), ("in place", rep, r)
            root = (rep + 1) % n_ranks
            rout = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.reduce([s.data_ptr() for s in send], [d.data_ptr() for d in rout], count, dt, op, root)
            exp = reduce_expected(inputs, dt, op, root, "ll")
            assert mg.canon_bytes(dt, rout[root].cpu().numpy()) == mg.canon_bytes(dt, exp), ("reduce", rep)
            bout = [torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()
            comm.broadcast([s.data_ptr() for s in send], [d.data_ptr() for d in bout], count, dt, root)
            exp = broadcast_expected(inputs, root)
            for r in range(n_ranks):
                assert bout[r].cpu().numpy().tobytes() == np.asarray(exp[r]).tobytes(), ("bcast", rep, r)
            per = count // n_ranks
            rs = [torch.zeros(per, dtype=send[0].dtype, device="cuda") for _ in range(n_ranks)]
            torch.cuda.synchronize()
            comm.reduce_scatter([s.data_ptr() for s in send], [d.data_ptr() for d in rs], per, dt, op)
            exp = reduce_scatter_expected([x[:per * n_ranks] for x in inputs], dt, op, "ll")
            for r in range(n_ranks):
                assert mg.canon_bytes(dt, rs[r].cpu().numpy()) == mg.canon_bytes(dt, exp[r]), ("rs", rep, r)
            ag = [torch.zeros(per * n_ranks, dtype=send[0].dtype, device="cuda") for _ in range(n_ranks)]
            torch.cuda.synchronize()
            comm.all_gather([s[:per].data_ptr() for s in send], [d.data_ptr() for d in ag], per, dt)
            exp = all_gather_expected([x[:per] for x in inputs])
            for r in range(n_ranks):
                assert ag[r].cpu().numpy().tobytes() == exp[r].tobytes(), ("ag", rep, r)
