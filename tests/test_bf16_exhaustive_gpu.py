"""Every bfloat16 bit pattern through the round-6 bf16 fold (nexr_types.hpp: gfx950's v_cvt_pk_bf16_f32 for
the round-to-nearest-even after every step, NaN canonicalised to 0x7fff once after the fold), against the
oracle's integer RNE with a NaN check per step (oracle/nexr_oracle.c, the reference's
__float2bfloat16_rn path, reduce_kernel.h:352-367), bit for bit — NaN payloads included, no canonical
comparison.

Operand a walks all 65,536 patterns; its partners are the same patterns rotated, so every pattern meets
subnormals, normals, both infinities and NaN payloads of both signs, and sums land on the subnormal /
normal boundary, on rounding ties and on overflow to infinity. Sum, Prod, Min, Max and PreMulSum, with
K = 2, 3 and 8 (a NaN produced mid-fold must stay NaN through the later steps and come out as 0x7fff)."""
import numpy as np
import pytest

import make_golden as mg
from test_reduce_copy_gpu import run_gpu

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ALL = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16)
SHIFTS = (1, 128, 255, 4099, 0x7f80, 0x8000, 0xff81)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _operands(k, shift):
    return [np.roll(ALL, (shift * s) % (1 << 16)).copy() for s in range(k)]


@pytest.mark.parametrize("k", [2, 3, 8])
@pytest.mark.parametrize("name,op", [("sum", mg.SUM), ("prod", mg.PROD), ("min", mg.MINMAX), ("max", mg.MINMAX),
                                     ("premulsum", mg.PREMULSUM)])
def test_every_bf16_pattern(nexr, oracle, dev, k, name, op):
    arg = mg.minmax_arg(mg.BF16, name == "max") if op == mg.MINMAX else 0
    pre = [0x3FC0 + 7 * s for s in range(k)] if op == mg.PREMULSUM else None  # 1.5, 1.5078, ... per source
    bad = []
    for shift in SHIFTS:
        srcs = _operands(k, shift)
        exp = oracle.reduce_copy(srcs, 1, mg.BF16, op, arg, pre, False)[0]
        got = run_gpu(nexr, srcs, 1, mg.BF16, op, arg, pre)[0]
        diff = np.nonzero(got.view(np.uint16) != exp.view(np.uint16))[0]
        if diff.size:
            i = int(diff[0])
            bad.append((shift, diff.size, [hex(int(s[i])) for s in srcs], hex(int(got.view(np.uint16)[i])),
                        hex(int(exp.view(np.uint16)[i]))))
    assert not bad, bad


def _ll_dev(a: np.ndarray):
    raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(raw.size + 64, dtype=torch.uint8, device="cuda")
    t[:raw.size] = torch.from_numpy(raw.copy()).cuda()
    return t


@pytest.mark.parametrize("n_recv", [1, 2])
@pytest.mark.parametrize("name,op", [("sum", mg.SUM), ("prod", mg.PROD), ("min", mg.MINMAX), ("max", mg.MINMAX),
                                     ("premulsum", mg.PREMULSUM)])
def test_every_bf16_pattern_ll_step(nexr, oracle, dev, n_recv, name, op):
    """The same through an LL step (nexrReduceCopyLL, peer-first folds, prims_ll.h:251-258): the user
    source plus one or two peers' lines, output to the user buffer and one send FIFO, against the
    oracle's LL restatement, bit for bit."""
    arg = (mg.minmax_arg(mg.BF16, name == "max") if op == mg.MINMAX
           else mg.float_scalar_bits(mg.BF16, 0.5) if op == mg.PREMULSUM else 0)
    n = ALL.size
    for shift in SHIFTS:
        srcs = _operands(1 + n_recv, shift)
        rflags = [300 + i for i in range(n_recv)]
        rlines = [oracle.make_ll_lines(srcs[1 + i], rflags[i]) for i in range(n_recv)]
        rc, odst, osends = oracle.reduce_copy_ll(srcs[0], True, rlines, rflags, True, 1, [77], n, mg.BF16, op, arg,
                                                 False)
        assert rc == 0
        d_src, d_recv = _ll_dev(srcs[0]), [_ll_dev(l) for l in rlines]
        d_dst = torch.zeros(n * 2 + 64, dtype=torch.uint8, device="cuda")
        d_send = torch.zeros(((n * 2 + 7) // 8) * 16 + 64, dtype=torch.uint8, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        nexr.reduce_copy_ll(d_src.data_ptr(), [t.data_ptr() for t in d_recv], rflags, d_dst.data_ptr(),
                            [d_send.data_ptr()], [77], n, mg.BF16, op, arg, True, False, status=status.data_ptr(),
                            timeout_us=2_000_000, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert int(status.item()) == 0
        got = d_dst.cpu().numpy()[:n * 2].view(np.uint16)
        exp = odst.view(np.uint16)
        diff = np.nonzero(got != exp)[0]
        assert diff.size == 0, (shift, diff.size, hex(int(got[diff[0]])), hex(int(exp[diff[0]])))
        g = d_send.cpu().numpy()[:osends[0].size]
        assert np.array_equal(g, osends[0].view(np.uint8)), shift
