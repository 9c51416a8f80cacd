"""GPU tests of the per-(datatype, fan-in) workgroup geometry (nexr_internal.h unroll_for/block_for):
fp16 with K = 8 runs 1024-lane workgroups with one pack per lane, every other shape 256 lanes with
four. Sizes straddle the 16 KiB trip (the one-shot body, the per-pack remainder loop and the scalar
edges), for the single launch and the batch launch, against the oracle bit for bit."""
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
