"""GPU parity tests: the HIP path (through the C ABI) against the golden vectors and the oracle.

Bar: bit-exact for every datatype (float32/float64 NaNs compared by class; half/bfloat16 bit-exact
including the canonical 0x7fff NaN). Sizes: every golden case, randomised mid-size cases for every
(datatype, op, K, M), the BASELINE.json configurations at full size, plus the edge cases the
reference's reduceCopy handles (unaligned heads/tails, pointers with different 16-B phases, byte
misalignment, in-place, K=M=8, empty calls).
"""
import ctypes
import hashlib
import os
import threading

import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

STORE_NP = mg.STORE


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _to_dev(arr: np.ndarray, offset_bytes: int = 0):
    """Device byte buffer holding arr at byte offset `offset_bytes` (plus guard bytes)."""
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    buf = torch.full((raw.size + offset_bytes + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    buf[offset_bytes:offset_bytes + raw.size] = torch.from_numpy(raw.copy()).cuda()
    return buf


def run_gpu(nexr, srcs, n_dsts, dt, op, arg=0, pre=None, post=False, src_off=None, dst_off=None, stream=None):
    n = srcs[0].size
    esz = mg.np.dtype(STORE_NP[dt]).itemsize
    src_off = src_off or [0] * len(srcs)
    dst_off = dst_off or [0] * n_dsts
    sbufs = [_to_dev(s, o) for s, o in zip(srcs, src_off)]
    dbufs = [torch.full((n * esz + o + 64,), 0x5A, dtype=torch.uint8, device="cuda") for o in dst_off]
    handle = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
    nexr.reduce_copy_ptrs([b.data_ptr() + o for b, o in zip(sbufs, src_off)],
                          [b.data_ptr() + o for b, o in zip(dbufs, dst_off)], n, dt, op, arg, pre, post, handle)
    torch.cuda.synchronize()
    outs = []
    for b, o in zip(dbufs, dst_off):
        host = b.cpu().numpy()
        # guard bytes around the output must be untouched
        assert (host[:o] == 0x5A).all() and (host[o + n * esz:] == 0x5A).all(), "write outside the destination"
        outs.append(host[o:o + n * esz].view(STORE_NP[dt]).copy())
    return outs


def same(dt, a, b):
    return mg.canon_bytes(dt, a) == mg.canon_bytes(dt, b)


def test_every_golden_vector_on_gpu(nexr, golden_cases, dev):
    bad = []
    for i, c in enumerate(golden_cases):
        srcs = mg.gen_inputs(c["dt"], c["k"], c["n"], c["seed"], c["special"])
        m = 1 + (i % 3)
        outs = run_gpu(nexr, srcs, m, c["dt"], c["op"], c["arg"], c["pre"], c["post"])
        for o in outs:
            if hashlib.sha256(mg.canon_bytes(c["dt"], o)).hexdigest() != c["sha256"]:
                bad.append((c["name"], mg.DT_NAMES[c["dt"]], c["k"], c["n"], c["special"], m))
                break
    assert not bad, f"{len(bad)} mismatches vs golden, first: {bad[:6]}"


OPS = [("sum", mg.SUM), ("prod", mg.PROD), ("min", mg.MINMAX), ("max", mg.MINMAX), ("premulsum", mg.PREMULSUM),
       ("sumpostdiv", mg.SUMPOSTDIV)]


def _case_args(dt, name, op, k, rng):
    arg, pre, post = 0, None, False
    if name in ("min", "max"):
        arg = mg.minmax_arg(dt, name == "max")
    if name == "premulsum":
        vals = [0.5, -1.25, 3.0, 0.125, 1.0, -0.75, 2.0, 0.3333333]
        npre = int(rng.integers(1, k + 1))
        pre = [mg.float_scalar_bits(dt, vals[s] if dt not in mg.INTS else s * 5 + 3) for s in range(npre)]
        post = True
    if name == "sumpostdiv":
        arg = (int(rng.integers(1, 9)) << 1) | int(dt in (mg.I8, mg.I32, mg.I64))
        post = True
    return arg, pre, post


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_matches_oracle_all_ops_k_m(nexr, oracle, dt, dev):
    rng = np.random.default_rng(dt)
    for name, op in OPS:
        if name == "sumpostdiv" and dt not in mg.INTS:
            continue
        for k in range(1, 9):
            n = int(rng.integers(1000, 70000))
            m = int(rng.choice([1, 2, 3, 8]))
            arg, pre, post = _case_args(dt, name, op, k, rng)
            srcs = mg.gen_inputs(dt, k, n, 777 + k * 31 + op, special=True)
            exp = oracle.reduce_copy(srcs, 1, dt, op, arg, pre, post)[0]
            for o in run_gpu(nexr, srcs, m, dt, op, arg, pre, post):
                assert same(dt, o, exp), (name, k, m, n)


@pytest.mark.parametrize("dt", [mg.I8, mg.F16, mg.F32, mg.F64, mg.BF16, mg.U64])
def test_unaligned_heads_tails_and_phases(nexr, oracle, dt, dev):
    esz = np.dtype(STORE_NP[dt]).itemsize
    rng = np.random.default_rng(100 + dt)
    for trial in range(16):
        k = int(rng.integers(1, 9))
        m = int(rng.integers(1, 4))
        n = int(rng.integers(1, 5000))
        srcs = mg.gen_inputs(dt, k, n, 4242 + trial, special=True)
        if trial < 4:    # same 16-B phase everywhere: head/body/tail split
            ph = int(rng.integers(0, 16 // esz)) * esz
            so, do = [ph] * k, [ph] * m
        elif trial < 8:  # different element-aligned phases: unaligned 16-B packs
            so = [int(rng.integers(0, 16 // esz)) * esz for _ in range(k)]
            do = [int(rng.integers(0, 16 // esz)) * esz for _ in range(m)]
        elif trial < 12:  # not even element-aligned (the ABI requires no alignment)
            so = [int(rng.integers(0, 16)) for _ in range(k)]
            do = [int(rng.integers(0, 16)) for _ in range(m)]
        else:            # anywhere in a 128-B line: the head that brings dst0 to a line boundary
            so = [int(rng.integers(0, 128)) // (esz if trial < 14 else 1) * (esz if trial < 14 else 1)
                  for _ in range(k)]
            do = [int(rng.integers(0, 128)) // (esz if trial < 14 else 1) * (esz if trial < 14 else 1)
                  for _ in range(m)]
        op, name = (mg.SUM, "sum") if trial % 2 == 0 else (mg.MINMAX, "max")
        arg = mg.minmax_arg(dt, True) if name == "max" else 0
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg)[0]
        for o in run_gpu(nexr, srcs, m, dt, op, arg, src_off=so, dst_off=do):
            assert same(dt, o, exp), (trial, so, do, n)


def test_in_place_dst_aliases_src0(nexr, oracle, dev):
    dt = mg.F32
    srcs = mg.gen_inputs(dt, 3, 100003, 5, special=False)
    exp = oracle.reduce_copy(srcs, 1, dt, mg.SUM)[0]
    bufs = [torch.from_numpy(s.copy()).cuda() for s in srcs]
    nexr.reduce_copy(bufs, [bufs[0]], mg.SUM)
    torch.cuda.synchronize()
    assert same(dt, bufs[0].cpu().numpy(), exp)


def test_torch_layer_and_streams(nexr, oracle, dev):
    s = torch.cuda.Stream()
    a = torch.randn(1 << 20, device="cuda")
    b = torch.randn(1 << 20, device="cuda")
    o = torch.empty_like(a)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        nexr.reduce_copy([a, b], [o], nexr.DevRedOp.Sum)
    s.synchronize()
    exp = oracle.reduce_copy([a.cpu().numpy(), b.cpu().numpy()], 1, mg.F32, mg.SUM)[0]
    assert same(mg.F32, o.cpu().numpy(), exp)


def test_hip_graph_capture_and_replay(nexr, oracle, dev):
    # nexrReduceCopy and nexrReduceCopyBatch are plain stream-ordered launches, so a HIP graph can
    # capture a chain of them (here: a K=2 sum feeding a K=3 max, plus a batch of small works) and
    # replay it on new data in place.
    n = 300_001
    a, b, c = (torch.randn(n, device="cuda") for _ in range(3))
    t = torch.empty_like(a)
    o = torch.empty_like(a)
    small_in = [torch.randn(1000 + i, device="cuda") for i in range(6)]
    small_out = [torch.empty_like(x) for x in small_in]
    max_arg = mg.minmax_arg(mg.F32, True)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nexr.reduce_copy([a, b], [t], nexr.DevRedOp.Sum)
        nexr.reduce_copy([t, c, a], [o], nexr.DevRedOp.MinMax, red_op_arg=max_arg)
        works = [nexr.make_work([x.data_ptr(), x.data_ptr()], [y.data_ptr()], x.numel())
                 for x, y in zip(small_in, small_out)]
        nexr.reduce_copy_batch(works, nexr.DataType.Float32, nexr.DevRedOp.Sum,
                               torch.cuda.current_stream().cuda_stream)
    for rep in range(3):
        for x in (a, b, c, *small_in):
            x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        an, bn, cn = (x.cpu().numpy() for x in (a, b, c))
        tn = oracle.reduce_copy([an, bn], 1, mg.F32, mg.SUM)[0]
        on = oracle.reduce_copy([tn, cn, an], 1, mg.F32, mg.MINMAX, max_arg)[0]
        assert same(mg.F32, t.cpu().numpy(), tn) and same(mg.F32, o.cpu().numpy(), on), rep
        for x, y in zip(small_in, small_out):
            xn = x.cpu().numpy()
            assert same(mg.F32, y.cpu().numpy(), oracle.reduce_copy([xn, xn], 1, mg.F32, mg.SUM)[0]), rep


def test_first_one_workgroup_per_cu_launch_inside_graph_capture():
    """The first launch of a kernel that reserves LDS for one workgroup per CU sets the kernel's
    dynamic-LDS attribute (once per device); in a fresh process that first launch is captured into a
    HIP graph, and the replays are exact (tests/graph_lds_worker.py)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    # NEXR_POLICY=3 (read once per process): the nt-store policy at this small size, where fp16 K = 8
    # launches 1 x 512 lanes held to one workgroup per CU by the LDS reservation (nexr_internal.h)
    p = subprocess.run([sys.executable, os.path.join(here, "graph_lds_worker.py")], capture_output=True, text=True,
                       timeout=180, env=dict(os.environ, NEXR_POLICY="3"))
    assert p.returncode == 0 and "graph replays exact" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]


def test_concurrent_callers_on_separate_streams(nexr, oracle, dev):
    n = 1 << 18
    jobs = []
    for t in range(4):
        srcs = mg.gen_inputs(mg.BF16, 4, n, 9000 + t, special=True)
        jobs.append((srcs, oracle.reduce_copy(srcs, 1, mg.BF16, mg.SUM)[0]))
    results = [None] * len(jobs)

    def work(i):
        st = torch.cuda.Stream()
        results[i] = run_gpu(nexr, jobs[i][0], 1, mg.BF16, mg.SUM, stream=st)[0]

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    [t.start() for t in ths]
    [t.join() for t in ths]
    for (srcs, exp), got in zip(jobs, results):
        assert same(mg.BF16, got, exp)


def test_host_staged_variant(nexr, oracle, dev):
    for dt, op, name in ((mg.F32, mg.SUM, "sum"), (mg.I8, mg.MINMAX, "min"), (mg.F16, mg.PROD, "prod")):
        srcs = mg.gen_inputs(dt, 2, 262144 + 3, 31 + dt, special=True)
        arg = mg.minmax_arg(dt, False) if name == "min" else 0
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg)[0]
        dsts = [np.zeros_like(srcs[0]) for _ in range(2)]
        nexr.reduce_copy_ptrs([s.ctypes.data for s in srcs], [d.ctypes.data for d in dsts], srcs[0].size, dt, op,
                              arg, host=True)
        for d in dsts:
            assert same(dt, d, exp)


def test_one_rank_launcher(nexr, oracle, dev):
    for dt in (mg.F32, mg.F16, mg.BF16, mg.F64, mg.I32, mg.U8):
        n = 131073  # a size where the reference's own grid split leaves a tail unwritten
        src = mg.gen_inputs(dt, 1, n, 55 + dt, special=True)[0]
        red = nexr.host_to_dev_red_op(nexr.RedOp.Avg, dt, 4)
        if dt in mg.INTS:  # integer Avg is SumPostDiv -> a plain copy on one rank (onerank.cc:50-55)
            assert red.op == nexr.DevRedOp.SumPostDiv
            exp = src
        else:
            assert red.op == nexr.DevRedOp.PreMulSum
            exp = oracle.reduce_copy([src], 1, dt, mg.PREMULSUM, red.scalarArg, [red.scalarArg], True)[0]
        s = _to_dev(src)
        d = torch.zeros_like(s)
        nexr.launch_one_rank(d.data_ptr(), s.data_ptr(), n, red, dt, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        esz = np.dtype(STORE_NP[dt]).itemsize
        assert same(dt, d.cpu().numpy()[:n * esz].view(STORE_NP[dt]), exp)
        # scalarArgIsPtr: the scalar is read from device memory (onerank.cc:32-42)
        if red.op == nexr.DevRedOp.PreMulSum:
            sc = torch.tensor([red.scalarArg], dtype=torch.int64).cuda()
            red2 = nexr.DevRedOpFull(red.op, red.proxyOp, 1, sc.data_ptr())
            d2 = torch.zeros_like(s)
            nexr.launch_one_rank(d2.data_ptr(), s.data_ptr(), n, red2, dt, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert same(dt, d2.cpu().numpy()[:n * esz].view(STORE_NP[dt]), exp)


def _full_size_check(nexr, oracle, dt, k, n, op, arg, threads=16):
    """Full-size BASELINE configuration: device-generated inputs, whole output vs the oracle."""
    g = torch.Generator(device="cuda")
    g.manual_seed(1234 + k + dt)
    esz = np.dtype(STORE_NP[dt]).itemsize
    if dt in mg.INTS:
        srcs = [torch.randint(0, 256, (n * esz,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    else:
        tdt = {mg.F32: torch.float32, mg.F16: torch.float16, mg.BF16: torch.bfloat16}[dt]
        srcs = [(torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt).view(torch.uint8) for _ in range(k)]
    dst = torch.empty(n * esz, dtype=torch.uint8, device="cuda")
    nexr.reduce_copy_ptrs([s.data_ptr() for s in srcs], [dst.data_ptr()], n, dt, op, arg, None, False,
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = [s.cpu().numpy().view(STORE_NP[dt]) for s in srcs]
    exp = oracle.reduce_copy(host, 1, dt, op, arg, threads=threads)[0]
    got = dst.cpu().numpy().view(STORE_NP[dt])
    assert same(dt, got, exp)


def test_config_c2_fp32_sum_k2_256mib(nexr, oracle, dev):
    _full_size_check(nexr, oracle, mg.F32, 2, 64 << 20, mg.SUM, 0)


@pytest.mark.parametrize("dt", [mg.F16, mg.BF16])
def test_config_c3_16bit_sum_k8_256mib(nexr, oracle, dt, dev):
    _full_size_check(nexr, oracle, dt, 8, 128 << 20, mg.SUM, 0)


@pytest.mark.parametrize("dt", [mg.I32, mg.I8])
@pytest.mark.parametrize("name", ["min", "max", "prod"])
def test_config_c4_int_sweep_k4_64mib(nexr, oracle, dt, name, dev):
    esz = np.dtype(STORE_NP[dt]).itemsize
    op = mg.PROD if name == "prod" else mg.MINMAX
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    _full_size_check(nexr, oracle, dt, 4, (64 << 20) // esz, op, arg)


def test_large_integer_sum_checksum_property(nexr, dev):
    # size-independent property at 1 GiB per buffer: sum of the output == sum of the input sums
    # (mod 2^64), computed on the device by torch independently of the kernel.
    n = (1 << 30) // 8
    a = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device="cuda")
    b = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device="cuda")
    o = torch.empty_like(a)
    nexr.reduce_copy([a, b], [o], nexr.DevRedOp.Sum)
    torch.cuda.synchronize()
    assert int(o.sum()) == int(a.sum() + b.sum())
    assert torch.equal(o, a + b)


def test_buffers_larger_than_4gib(nexr, dev):
    # 64-bit offsets end to end: 4.5 Gi int8 elements per buffer (13.5 GiB in HBM), K=2 sum with
    # wrap-around, checked on the device against torch's own uint8 add.
    n = (9 << 30) // 2
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    b = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    o = torch.empty_like(a)
    nexr.reduce_copy([a, b], [o], nexr.DevRedOp.Sum, datatype=nexr.DataType.Uint8)
    torch.cuda.synchronize()
    assert torch.equal(o, a + b)
    del a, b, o
    torch.cuda.empty_cache()


def test_mixed_phases_beyond_4_gib(nexr, dev):
    """Advisor r1, on hardware (round 1's per-element path for mixed 16-B phases needed more work items
    than HIP launches here; round 2 moves such calls as unaligned 16-B packs): 2^32 + 4099 uint8
    elements with src1 one byte off src0's phase, the grid within HIP's work-item limit."""
    n = (1 << 32) + 4099
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    braw = torch.randint(0, 256, (n + 1,), dtype=torch.uint8, device="cuda", generator=g)
    b = braw[1:]  # 16-B phase 1 against a's phase 0: no common alignment
    o = torch.empty_like(a)
    info = nexr.query_launch([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n, nexr.DataType.Uint8)
    assert info.unaligned == 1 and info.grid * info.block <= 0xFFFFFFFF < n
    nexr.reduce_copy([a, b], [o], nexr.DevRedOp.Sum, datatype=nexr.DataType.Uint8)
    torch.cuda.synchronize()
    assert torch.equal(o, a + b)
    del a, braw, b, o
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dt,n,op,name", [(mg.F32, 5_000_003, mg.SUM, "sum"), (mg.I8, 30_000_001, mg.MINMAX, "max"),
                                          (mg.BF16, 9_000_017, mg.PROD, "prod")])
def test_host_staged_pipeline_multi_chunk(nexr, oracle, dt, n, op, name, dev):
    # several 8 MiB chunks with a ragged last one; copy-in of chunk c overlaps copy-out of c-1
    srcs = mg.gen_inputs(dt, 3, n, 61 + dt, special=True)
    arg = mg.minmax_arg(dt, True) if name == "max" else 0
    exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=16)[0]
    dsts = [np.zeros_like(srcs[0]) for _ in range(2)]
    nexr.reduce_copy_ptrs([s.ctypes.data for s in srcs], [d.ctypes.data for d in dsts], n, dt, op, arg, host=True)
    for d in dsts:
        assert same(dt, d, exp)


def test_host_staging_rings_are_pooled_not_per_thread(nexr, oracle, dev):
    """Callers such as the emulated collectives run every call's ranks on fresh threads. Each
    host-staged call checks a staging ring out of a process-wide pool and returns it, so 40 calls
    from 40 short-lived threads (and 8 at once) reuse a bounded set of rings: device memory must not
    grow by one ring (here 2 x 3 x 4 MiB) per thread."""
    n = 1_000_003
    srcs = mg.gen_inputs(mg.F32, 2, n, 4242, special=True)
    exp = oracle.reduce_copy(srcs, 1, mg.F32, mg.SUM)[0]
    sp = [s.ctypes.data for s in srcs]
    errors = []

    def call():
        try:
            torch.cuda.set_device(0)
            d = np.zeros_like(srcs[0])
            nexr.reduce_copy_ptrs(sp, [d.ctypes.data], n, mg.F32, mg.SUM, host=True)
            if not same(mg.F32, d, exp):
                errors.append("mismatch")
        except Exception as e:  # noqa: BLE001 - collected and asserted below
            errors.append(repr(e))

    def run_threads(k):
        ths = [threading.Thread(target=call) for _ in range(k)]
        [t.start() for t in ths]
        [t.join() for t in ths]

    run_threads(1)  # the pool's first ring
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    for _ in range(40):
        run_threads(1)
    for _ in range(3):
        run_threads(8)
    torch.cuda.synchronize()
    grown = free0 - torch.cuda.mem_get_info(0)[0]
    assert not errors, errors[:3]
    ring = 2 * 3 * (4 << 20)
    # at most the 7 extra rings the 8-way rounds need (one ring per concurrent call), never one per thread
    assert grown <= 8 * ring, f"device memory grew by {grown / 2**20:.0f} MiB over 64 host-staged threads"


def test_host_zero_copy_pinned_buffers(nexr, oracle, dev):
    # pinned (device-mapped) host buffers: the kernel reads/writes them in place over PCIe;
    # interior pointers (offset into the allocation) and a pinned/pageable mix (-> staged) too.
    n = 3_000_001
    srcs = mg.gen_inputs(mg.F16, 4, n, 808, special=True)
    exp = oracle.reduce_copy(srcs, 1, mg.F16, mg.SUM, threads=16)[0]
    pin = [torch.empty(n * 2 + 64, dtype=torch.uint8).pin_memory() for _ in range(6)]
    for p, s in zip(pin, srcs):
        p[32:32 + n * 2].copy_(torch.from_numpy(s.view(np.uint8)))
    sp = [p.data_ptr() + 32 for p in pin[:4]]
    dp = [pin[4].data_ptr() + 32, pin[5].data_ptr() + 32]
    nexr.reduce_copy_ptrs(sp, dp, n, mg.F16, mg.SUM, host=True)
    for p in pin[4:]:
        assert same(mg.F16, p[32:32 + n * 2].numpy().view(np.uint16), exp)
    pageable = np.zeros_like(srcs[0])
    nexr.reduce_copy_ptrs(sp, [pinned for pinned in dp[:1]] + [pageable.ctypes.data], n, mg.F16, mg.SUM, host=True)
    assert same(mg.F16, pageable, exp)


@pytest.mark.parametrize("mask", [0b00001, 0b00110, 0b01011, 0b10000, 0b11100, 0b01111, 0b10101])
def test_host_partially_pinned_buffers(nexr, oracle, dev, mask):
    """Pinned and pageable host buffers in one call (e.g. pinned FIFOs beside pageable user buffers):
    the kernel reads/writes the pinned ones in place and only the pageable ones are staged. Bit i of
    `mask` pins buffer i of [src0, src1, src2, dst0, dst1]; 3 chunks of 8 MiB plus a ragged one."""
    n = 6_000_011
    dt = mg.F32
    srcs = mg.gen_inputs(dt, 3, n, 900 + mask, special=True)
    exp = oracle.reduce_copy(srcs, 1, dt, mg.SUM, threads=16)[0]
    bufs, keep = [], []
    for i in range(5):
        if mask >> i & 1:
            t = torch.zeros(n, dtype=torch.float32).pin_memory()
            if i < 3:
                t.copy_(torch.from_numpy(srcs[i]))
            keep.append(t)
            bufs.append((t.data_ptr(), lambda t=t: t.numpy()))
        else:
            a = srcs[i].copy() if i < 3 else np.zeros(n, np.float32)
            keep.append(a)
            bufs.append((a.ctypes.data, lambda a=a: a))
    nexr.reduce_copy_ptrs([b[0] for b in bufs[:3]], [b[0] for b in bufs[3:]], n, dt, mg.SUM, host=True)
    for b in bufs[3:]:
        assert same(dt, b[1](), exp)
    # in place on src0, whatever its kind
    nexr.reduce_copy_ptrs([b[0] for b in bufs[:3]], [bufs[0][0]], n, dt, mg.SUM, host=True)
    assert same(dt, bufs[0][1](), exp)


def test_random_fuzz_against_oracle(nexr, oracle, dev):
    # 300 random (datatype, op, K, M, n, per-pointer offsets, pre/post) cases, special values on
    rng = np.random.default_rng(20261015)
    ops = [("sum", mg.SUM), ("prod", mg.PROD), ("min", mg.MINMAX), ("max", mg.MINMAX), ("premulsum", mg.PREMULSUM),
           ("sumpostdiv", mg.SUMPOSTDIV)]
    for case in range(300):
        dt = int(rng.choice(sorted(mg.DT_NAMES)))
        name, op = ops[int(rng.integers(0, len(ops)))]
        if name == "sumpostdiv" and dt not in mg.INTS:
            name, op = "sum", mg.SUM
        k = int(rng.integers(1, 9))
        m = int(rng.integers(1, 9))
        n = int(rng.choice([1, 2, 7, 15, 16, 17, 255, 1023, 4097, 65535, 300_001]))
        esz = np.dtype(mg.STORE[dt]).itemsize
        mode = int(rng.integers(0, 3))
        if mode == 0:
            so, do = [0] * k, [0] * m
        elif mode == 1:
            ph = int(rng.integers(0, 16 // esz)) * esz
            so, do = [ph] * k, [ph] * m
        else:
            so = [int(rng.integers(0, 16)) for _ in range(k)]
            do = [int(rng.integers(0, 16)) for _ in range(m)]
        arg, pre, post = _case_args(dt, name, op, k, rng)
        srcs = mg.gen_inputs(dt, k, n, 5000 + case, special=True)
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, pre, post)[0]
        for o in run_gpu(nexr, srcs, m, dt, op, arg, pre, post, src_off=so, dst_off=do):
            assert same(dt, o, exp), (case, mg.DT_NAMES[dt], name, k, m, n, so, do)


@pytest.mark.parametrize("offs", [(0, 4, 0), (4, 0, 12), (1, 3, 5), (0, 0, 1)])
def test_large_misaligned_streams(nexr, dev, offs):
    """256 MiB per buffer (768 MiB streamed: non-temporal loads and stores) with the sources and the
    destination at the given byte offsets, element-aligned or not: the body's unaligned 16-B packs
    under the streaming policy, checked bit for bit against torch's fp32 add, guard bytes intact."""
    n = 64 << 20
    nb = n * 4
    g = torch.Generator(device="cuda")
    g.manual_seed(sum(offs) + 5)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g) * 2 - 1
    raw = [torch.full((nb + 256,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(3)]
    raw[0][offs[0]:offs[0] + nb] = a.view(torch.uint8)
    raw[1][offs[1]:offs[1] + nb] = b.view(torch.uint8)
    info = nexr.query_launch([raw[0].data_ptr() + offs[0], raw[1].data_ptr() + offs[1]],
                             [raw[2].data_ptr() + offs[2]], n, nexr.DataType.Float32)
    assert info.policy == 3 and info.unaligned == int(len({o % 16 for o in offs}) > 1)
    nexr.reduce_copy_ptrs([raw[0].data_ptr() + offs[0], raw[1].data_ptr() + offs[1]], [raw[2].data_ptr() + offs[2]],
                          n, nexr.DataType.Float32, nexr.DevRedOp.Sum,
                          stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = raw[2][offs[2]:offs[2] + nb].clone().view(torch.float32)
    assert torch.equal(out.view(torch.int32), (a + b).view(torch.int32))
    assert bool((raw[2][:offs[2]] == 0x5A).all()) and bool((raw[2][offs[2] + nb:] == 0x5A).all())
    del a, b, raw, out
    torch.cuda.empty_cache()
