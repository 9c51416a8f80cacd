"""GPU tests of the per-(datatype, fan-in, cache policy) workgroup geometry (nexr_internal.h
unroll_for/block_for): fp16/bf16 with K = 8 run 1024-lane workgroups with one pack per lane; K = 4
runs 2 packs x 512 lanes once a call streams 64-512 MiB and 1 x 1024 beyond (fp16 excepted); every
other shape 256 lanes with four. Sizes straddle the 16 KiB trip (the one-shot body, the per-pack
remainder loop and the scalar edges), for the single launch and the batch launch, against the oracle
bit for bit."""
import numpy as np
import pytest

import make_golden as mg

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TRIP_ELEMS_F16 = 1024 * 8  # one trip = 1024 packs of 8 halves


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _run(nexr, srcs, dt, op, arg, offs=None):
    n = srcs[0].size
    esz = srcs[0].itemsize
    offs = offs or [0] * (len(srcs) + 1)
    bufs = []
    for s, o in zip(srcs, offs):
        b = torch.zeros(n * esz + o + 64, dtype=torch.uint8, device="cuda")
        b[o:o + n * esz] = torch.from_numpy(s.view(np.uint8).copy()).cuda()
        bufs.append(b)
    out = torch.full((n * esz + offs[-1] + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    nexr.reduce_copy_ptrs([b.data_ptr() + o for b, o in zip(bufs, offs)], [out.data_ptr() + offs[-1]], n, dt, op, arg,
                          None, False, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    assert (host[:offs[-1]] == 0x5A).all() and (host[offs[-1] + n * esz:] == 0x5A).all()
    return host[offs[-1]:offs[-1] + n * esz].view(srcs[0].dtype)


@pytest.mark.parametrize("n", [1, 7, 8, TRIP_ELEMS_F16 - 8, TRIP_ELEMS_F16, TRIP_ELEMS_F16 + 1,
                               3 * TRIP_ELEMS_F16 + 5, 100 * TRIP_ELEMS_F16 + 8 * 37 + 3])
@pytest.mark.parametrize("op,name", [(mg.SUM, "sum"), (mg.PROD, "prod"), (mg.MINMAX, "min")])
def test_f16_k8_geometry_edges(nexr, oracle, dev, n, op, name):
    srcs = mg.gen_inputs(mg.F16, 8, n, 9000 + n % 977, special=True)
    arg = mg.minmax_arg(mg.F16, False) if op == mg.MINMAX else 0
    exp = oracle.reduce_copy(srcs, 1, mg.F16, op, arg)[0]
    assert mg.canon_bytes(mg.F16, _run(nexr, srcs, mg.F16, op, arg)) == mg.canon_bytes(mg.F16, exp)
    # same 16-B phase on every pointer (head/body/tail split), then mixed phases (scalar path)
    for offs in ([6] * 9, [0, 2, 4, 6, 8, 10, 12, 14, 2]):
        assert mg.canon_bytes(mg.F16, _run(nexr, srcs, mg.F16, op, arg, offs)) == mg.canon_bytes(mg.F16, exp)


def test_f16_k8_in_a_batch_beside_other_shapes(nexr, oracle, dev):
    # a batch mixing K = 8 works (1024-lane geometry) with K = 2 works (256-lane geometry)
    rng = np.random.default_rng(5)
    works, expect, outs, keep = [], [], [], []
    for i in range(9):
        k = 8 if i % 2 == 0 else 2
        n = int(rng.integers(1, 5 * TRIP_ELEMS_F16))
        srcs = mg.gen_inputs(mg.F16, k, n, 300 + i, special=True)
        ts = [torch.from_numpy(s.copy()).cuda() for s in srcs]
        o = torch.zeros(n, dtype=ts[0].dtype, device="cuda")
        keep += ts
        outs.append(o)
        works.append(nexr.make_work([t.data_ptr() for t in ts], [o.data_ptr()], n))
        expect.append(oracle.reduce_copy(srcs, 1, mg.F16, mg.SUM)[0])
    nexr.reduce_copy_batch(works, mg.F16, mg.SUM, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for o, e in zip(outs, expect):
        assert mg.canon_bytes(mg.F16, o.cpu().numpy()) == mg.canon_bytes(mg.F16, e)


# ---- K = 4: the geometry follows the cache policy -------------------------------------------------------
MIB = 1 << 20


@pytest.mark.parametrize("dt,op,name,buf_mib", [
    (mg.I8, mg.MINMAX, "min", 16), (mg.I32, mg.PROD, "prod", 16), (mg.F32, mg.SUM, "sum", 13),  # 2 x 512 / 4 x 256
    (mg.U32, mg.MINMAX, "max", 104), (mg.BF16, mg.SUM, "sum", 104),                              # 1 x 1024 / 2 x 512
    (mg.F16, mg.SUM, "sum", 104)])                                                               # 4 x 256
def test_k4_policy_geometries_edges(nexr, oracle, dev, dt, op, name, buf_mib):
    esz = np.dtype(mg.STORE[dt]).itemsize
    base = buf_mib * MIB // esz
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    for n, offs in ((base, None), (base + 16 // esz * 1024 * 3 + 5, None), (base - 7, [esz] * 5),
                    (base + 1, [0, esz, 0, 2 * esz, esz])):
        srcs = mg.gen_inputs(dt, 4, n, 4400 + n % 1013, special=True)
        info = nexr.query_launch([0x100000 * (i + 1) + (offs[i] if offs else 0) for i in range(4)],
                                 [0x900000 + (offs[4] if offs else 0)], n, dt)
        if offs is None or len(set(offs)) == 1:
            if info.policy == 1:
                assert info.block == (256 if esz == 4 else 512)
            else:
                assert info.block == {mg.F16: 256, mg.BF16: 512}.get(dt, 1024)
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=16)[0]
        got = _run(nexr, srcs, dt, op, arg, offs)
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp), (n, offs)
        del srcs, exp, got
        torch.cuda.empty_cache()


def test_k4_batch_at_the_c4_policy(nexr, oracle, dev):
    """A batch of K = 4 works streaming more than 64 MiB in total launches the 2 x 512 geometry;
    each work's bytes must match the oracle, as must K = 2 works batched beside them (4 x 256)."""
    rng = np.random.default_rng(44)
    works, expect, outs, keep = [], [], [], []
    for i in range(6):
        k = 4 if i % 3 else 2
        n = int(rng.integers(2 * MIB, 4 * MIB))
        srcs = mg.gen_inputs(mg.I8, k, n, 700 + i, special=True)
        ts = [torch.from_numpy(s.copy()).cuda() for s in srcs]
        o = torch.zeros(n, dtype=ts[0].dtype, device="cuda")
        keep += ts
        outs.append(o)
        arg = mg.minmax_arg(mg.I8, False)
        works.append(nexr.make_work([t.data_ptr() for t in ts], [o.data_ptr()], n, arg))
        expect.append(oracle.reduce_copy(srcs, 1, mg.I8, mg.MINMAX, arg)[0])
    big = [torch.from_numpy(s.copy()).cuda() for s in mg.gen_inputs(mg.I8, 4, 16 * MIB, 799, special=True)]
    ob = torch.zeros(16 * MIB, dtype=big[0].dtype, device="cuda")
    works.append(nexr.make_work([t.data_ptr() for t in big], [ob.data_ptr()], 16 * MIB, mg.minmax_arg(mg.I8, False)))
    expect.append(oracle.reduce_copy([t.cpu().numpy() for t in big], 1, mg.I8, mg.MINMAX, mg.minmax_arg(mg.I8, False))[0])
    outs.append(ob)
    nexr.reduce_copy_batch(works, mg.I8, mg.MINMAX, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for o, e in zip(outs, expect):
        assert mg.canon_bytes(mg.I8, o.cpu().numpy()) == mg.canon_bytes(mg.I8, e)


def test_k4_geometry_random_large_calls(nexr, oracle, dev):
    """Eight random K = 4 calls in both new regimes (13-140 MiB per buffer: 64-700 MiB streamed),
    random datatype and op, random pointer phases (shared: the 2x512 / 1x1024 body; mixed: the
    element path at the same geometry), M = 1 or 2, against the oracle."""
    rng = np.random.default_rng(4242)
    ops = [(mg.SUM, "sum"), (mg.PROD, "prod"), (mg.MINMAX, "min"), (mg.MINMAX, "max")]
    for case in range(8):
        dt = int(rng.choice([mg.I8, mg.U8, mg.I32, mg.U32, mg.I64, mg.F16, mg.F32, mg.F64, mg.BF16]))
        op, name = ops[int(rng.integers(0, len(ops)))]
        esz = np.dtype(mg.STORE[dt]).itemsize
        n = int(rng.integers(13 * MIB, 140 * MIB)) // esz
        shared = bool(rng.integers(0, 2))
        ph = int(rng.integers(0, 16 // esz)) * esz
        offs = [ph] * 5 if shared else [int(rng.integers(0, 16 // esz)) * esz for _ in range(5)]
        arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
        srcs = mg.gen_inputs(dt, 4, n, 9100 + case, special=True)
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=16)[0]
        got = _run(nexr, srcs, dt, op, arg, offs)
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp), (case, mg.DT_NAMES[dt], name, n, offs)
        del srcs, exp, got
        torch.cuda.empty_cache()


# ---- K >= 6 under the nt-store policy: one pack x 512 lanes, one workgroup per CU (round 5) -----------
@pytest.mark.parametrize("dt,k,op,name,buf_mib", [(mg.F32, 6, mg.SUM, "sum", 88), (mg.I32, 8, mg.MINMAX, "max", 60),
                                                  (mg.F64, 7, mg.SUM, "sum", 68)])
def test_wide_fan_in_nt_store_geometry_edges(nexr, oracle, dev, dt, k, op, name, buf_mib):
    esz = np.dtype(mg.STORE[dt]).itemsize
    base = buf_mib * MIB // esz
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    for n, offs in ((base + 16 // esz * 1024 * 2 + 3, None), (base - 5, [esz] * (k + 1))):
        srcs = mg.gen_inputs(dt, k, n, 5100 + n % 1013, special=True)
        info = nexr.query_launch([0x1000000 * (i + 1) + (offs[i] if offs else 0) for i in range(k)],
                                 [0x9000000 + (offs[k] if offs else 0)], n, dt)
        assert (info.policy, info.block, info.packsPerLane) == (3, 512, 1), (n, offs)
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=16)[0]
        got = _run(nexr, srcs, dt, op, arg, offs)
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp), (n, offs)
        del srcs, exp, got
        torch.cuda.empty_cache()


@pytest.mark.parametrize("dt,k", [(mg.F16, 8), (mg.BF16, 6)])
def test_16bit_wide_fan_in_nt_store_geometry(nexr, oracle, dev, dt, k):
    """fp16 K = 8 and bf16 K >= 6 at >= 512 MiB streamed run 512 lanes (bf16 since round 6's hardware
    RNE), one pack per lane at one workgroup per CU; a size just past a trip boundary, against the oracle."""
    n = 40 * MIB + 8 * 512 * 2 + 3  # 80 MiB per buffer: >= 512 MiB streamed for K >= 6
    srcs = mg.gen_inputs(dt, k, n, 6100 + k, special=True)
    info = nexr.query_launch([0x1000000 * (i + 1) for i in range(k)], [0x9000000], n, dt)
    assert (info.policy, info.block, info.packsPerLane) == (3, 512, 1)
    exp = oracle.reduce_copy(srcs, 1, dt, mg.SUM, 0, threads=16)[0]
    assert mg.canon_bytes(dt, _run(nexr, srcs, dt, mg.SUM, 0)) == mg.canon_bytes(dt, exp)


# ---- K <= 2 with M <= 2: nt stores from 96 MiB streamed (round 5, nexr_api.cpp pickPolicy) ---------------
def _run_m(nexr, srcs, m, dt, op, arg, offs):
    n, esz = srcs[0].size, srcs[0].itemsize
    bufs = []
    for s, o in zip(srcs, offs):
        b = torch.zeros(n * esz + o + 64, dtype=torch.uint8, device="cuda")
        b[o:o + n * esz] = torch.from_numpy(s.view(np.uint8).copy()).cuda()
        bufs.append(b)
    douts = offs[len(srcs):]
    outs = [torch.full((n * esz + o + 64,), 0x5A, dtype=torch.uint8, device="cuda") for o in douts]
    nexr.reduce_copy_ptrs([b.data_ptr() + o for b, o in zip(bufs, offs)], [t.data_ptr() + o for t, o in zip(outs, douts)],
                          n, dt, op, arg, None, False, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = []
    for t, o in zip(outs, douts):
        host = t.cpu().numpy()
        assert (host[:o] == 0x5A).all() and (host[o + n * esz:] == 0x5A).all(), "write outside a destination"
        got.append(host[o:o + n * esz].view(srcs[0].dtype))
    return got


@pytest.mark.parametrize("dt,k,m,op,name,buf_mib", [(mg.F32, 1, 1, mg.SUM, "sum", 49), (mg.I8, 1, 2, mg.MINMAX, "max", 33),
                                                    (mg.F32, 2, 2, mg.SUM, "sum", 25), (mg.BF16, 2, 2, mg.PROD, "prod", 26),
                                                    (mg.F16, 1, 4, mg.SUM, "sum", 20), (mg.I32, 3, 2, mg.MINMAX, "min", 20),
                                                    (mg.F32, 2, 6, mg.SUM, "sum", 13), (mg.U8, 3, 5, mg.MINMAX, "max", 13),
                                                    (mg.F32, 2, 7, mg.SUM, "sum", 11), (mg.BF16, 3, 7, mg.SUM, "sum", 10)])
def test_small_fan_in_nt_store_policy_edges(nexr, oracle, dev, dt, k, m, op, name, buf_mib):
    """Copies (K = 1), the ring's two-destination steps and the tree's K = 1 M = 4 / K = 3 M = 2 steps
    just past 96 MiB streamed launch the nt-store policy at the default 4 x 256 shape; whole trips, a remainder plus edges, and mixed 16-B phases
    against the oracle bit for bit, every destination, guard bytes intact."""
    esz = np.dtype(mg.STORE[dt]).itemsize
    base = buf_mib * MIB // esz
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    mixed = [(i * 3) % 16 // esz * esz for i in range(k + m)]
    for n, offs in ((base, [0] * (k + m)), (base + 16 // esz * 1024 * 3 + 5, [esz] * (k + m)), (base - 7, mixed)):
        info = nexr.query_launch([0x1000000 * (i + 1) + offs[i] for i in range(k)],
                                 [0x90000000 + 0x1000000 * d + offs[k + d] for d in range(m)], n, dt)
        assert (info.policy, info.block, info.packsPerLane) == (3, 256, 4), (n, offs)
        srcs = mg.gen_inputs(dt, k, n, 5100 + n % 1009, special=True)
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=16)[0]
        for got in _run_m(nexr, srcs, m, dt, op, arg, offs):
            assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp), (n, offs)
        del srcs, exp
        torch.cuda.empty_cache()


@pytest.mark.parametrize("dt,k,op,name,buf_mib", [(mg.F32, 5, mg.SUM, "sum", 88), (mg.BF16, 5, mg.SUM, "sum", 88),
                                                  (mg.I8, 5, mg.MINMAX, "min", 88)])
def test_k5_nt_store_geometry_edges(nexr, oracle, dev, dt, k, op, name, buf_mib):
    """K = 5 under the nt-store policy runs one pack x 1024 lanes at one workgroup per CU, as K = 4 does
    (round 5), and bf16 one pack x 512 lanes at two per CU (round 6); whole trips, a remainder plus
    edges, and mixed phases against the oracle."""
    esz = np.dtype(mg.STORE[dt]).itemsize
    base = buf_mib * MIB // esz
    arg = mg.minmax_arg(dt, name == "max") if op == mg.MINMAX else 0
    for n, offs in ((base, None), (base + 16 // esz * 1024 * 3 + 5, None), (base - 7, [esz * (i % 2) for i in range(k + 1)])):
        info = nexr.query_launch([0x1000000 * (i + 1) + (offs[i] if offs else 0) for i in range(k)],
                                 [0x90000000 + (offs[k] if offs else 0)], n, dt)
        assert (info.policy, info.block, info.packsPerLane) == (3, 512 if dt == mg.BF16 else 1024, 1), (n, offs)
        srcs = mg.gen_inputs(dt, k, n, 5300 + n % 1013, special=True)
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=16)[0]
        got = _run(nexr, srcs, dt, op, arg, offs)
        assert mg.canon_bytes(dt, got) == mg.canon_bytes(dt, exp), (n, offs)
        del srcs, exp, got
        torch.cuda.empty_cache()


def test_lds_reserving_launch_on_another_devices_stream(nexr, oracle):
    """Advisor r5 (low): the one-workgroup-per-CU shapes launch with 120 KiB of dynamic LDS, which the
    kernel must be allowed first; HIP applies that attribute on the CURRENT device, so the library sets
    it on the stream's device. First launch of a fresh (datatype, K, policy) on a device-1 stream while
    device 0 is current: exact (needs two GPUs)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    n = (600 << 20) // 9 // 2 // 16 * 16  # fp16 K = 8, > 512 MiB streamed: nt stores, 1 x 512 at one per CU
    srcs = mg.gen_inputs(mg.F16, 8, 4099, 9100, special=True)
    exp = oracle.reduce_copy(srcs, 1, mg.F16, mg.SUM, 0)[0]
    torch.cuda.set_device(0)
    d1 = torch.device("cuda:1")
    reps = n // 4099 + 1
    bufs = [torch.from_numpy(np.tile(s, reps)[:n].view(np.uint8).copy()).to(d1) for s in srcs]
    out = torch.full((n * 2,), 0x5A, dtype=torch.uint8, device=d1)
    s1 = torch.cuda.Stream(device=d1)
    nexr.reduce_copy_ptrs([b.data_ptr() for b in bufs], [out.data_ptr()], n, mg.F16, mg.SUM, 0, None, False,
                          s1.cuda_stream)
    s1.synchronize()
    assert torch.cuda.current_device() == 0
    got = out[:4099 * 2].cpu().numpy().view(np.float16)
    assert mg.canon_bytes(mg.F16, got) == mg.canon_bytes(mg.F16, exp)
