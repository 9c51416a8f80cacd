"""nexrReduceCopyHost's zero-copy path for every datatype x op x K (1-8) x M (1-8).

A launch that touches host memory runs a capped grid (hostGrid, 32 workgroups, nexr_api.cpp), so
every workgroup loops over several trips, a schedule device launches (one-shot grids) do not use, and
every access crosses PCIe. Buffers lie in one nexrHostMemAlloc region at byte offsets that give head
and tail edges and mixed 16-B phases; sizes give up to 8 trips per workgroup. Results must equal the
oracle bit for bit (NaNs by class, as everywhere), guard bytes around every destination must be
intact, and every call must have run zero-copy from the registration cache with no runtime pointer
query (nexrGetHostPathStats)."""
import ctypes

import numpy as np
import pytest

import make_golden as mg
from test_reduce_copy_gpu import OPS, _case_args, same

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

REGION = 48 << 20
GUARD = 0x5A


@pytest.fixture(scope="module")
def region(nexr):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    addr = nexr.host_mem_alloc(REGION)
    view = np.ctypeslib.as_array((ctypes.c_uint8 * REGION).from_address(addr))
    yield addr, view
    nexr.host_mem_free(addr)


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_zero_copy_every_op_k_m(nexr, oracle, region, dt):
    addr, view = region
    esz = np.dtype(mg.STORE[dt]).itemsize
    rng = np.random.default_rng(900 + dt)
    nexr.host_path_stats(reset=True)
    calls = 0
    for name, op in OPS:
        if name == "sumpostdiv" and dt not in mg.INTS:
            continue
        for k in range(1, 9):
            m = [1, 2, 3, 8][(k + op) % 4]
            # 32 workgroups x 16 KiB trips: 1-4 MiB per buffer is 2-8 trips per workgroup
            n = int(rng.integers(1 << 20, 4 << 20)) // esz // max(1, (k + m) // 4) + int(rng.integers(0, 97))
            arg, pre, post = _case_args(dt, name, op, k, rng)
            srcs = mg.gen_inputs(dt, k, n, 31 * dt + 7 * k + op, special=True)
            exp = oracle.reduce_copy(srcs, 1, dt, op, arg, pre, post, threads=8)[0]
            same_phase = k % 2 == 0
            ph = int(rng.integers(0, 16))
            cur, sp, dp, guard_lo = 0, [], [], []
            for s in srcs:  # sources: each at its own phase, or all at one
                off = ph if same_phase else int(rng.integers(0, 16))
                raw = s.view(np.uint8).reshape(-1)
                view[cur + off:cur + off + raw.size] = raw
                sp.append(cur + off)
                cur += (off + raw.size + 255) & ~127
            for _ in range(m):
                off = ph if same_phase else int(rng.integers(0, 16))
                view[cur:cur + off + n * esz + 64] = GUARD
                guard_lo.append(cur)
                dp.append(cur + off)
                cur += (off + n * esz + 64 + 255) & ~127
            assert cur <= REGION, (k, m, n)
            nexr.reduce_copy_ptrs([addr + p for p in sp], [addr + p for p in dp], n, dt, op, arg, pre, post,
                                  host=True)
            calls += 1
            for lo, p in zip(guard_lo, dp):
                got = view[p:p + n * esz].copy().view(mg.STORE[dt])
                assert same(dt, got, exp), (mg.DT_NAMES[dt], name, k, m, n)
                assert (view[lo:p] == GUARD).all(), ("write before the start", name, k, m)
                assert (view[p + n * esz:p + n * esz + 64] == GUARD).all(), ("write past the end", name, k, m)
    st = nexr.host_path_stats(reset=True)
    assert st["calls"] == calls and st["zeroCopyCalls"] == calls, st
    assert st["pointerQueries"] == 0, st
