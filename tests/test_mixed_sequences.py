"""Random sequences of every emulated collective on ONE communicator (CPU, the oracle serving every
reduceCopy): ring AllReduce / ReduceScatter / AllGather / Reduce / Broadcast and tree AllReduce (and,
with the opt-in extras library, grouped Send/Recv) share links and step counters across calls, with
different slice geometries (1-step and 2-step slices), so every transition between them is
exercised: round-up with credit return, FIFO wrap. Integer sums make the expected result plain
arithmetic, independent of fold order."""
import ctypes
import importlib

import numpy as np
import pytest


@pytest.fixture(scope="module")
def ring(nexr):
    return importlib.import_module("nex-nccl_amd.ring")


@pytest.fixture(scope="module")
def fn(oracle):
    return ctypes.cast(oracle.lib().oracle_reduce_copy_fn, ctypes.c_void_p).value


U32 = 3
KINDS = ("ar", "rs", "ag", "reduce", "bcast", "tree")
EXTRA_KINDS = ("sendrecv",)  # the opt-in extras library (include/nexr_extras.h)


def _ptrs(arrs):
    return [a.ctypes.data for a in arrs]


@pytest.mark.parametrize("n,seed", [(2, 1), (2, 2), (2, 7), (3, 3), (3, 8), (4, 4), (4, 9), (5, 5), (6, 10), (7, 11), (8, 6),
                                    (13, 12)])
@pytest.mark.parametrize("extras", [False, True])
def test_random_collective_sequences(ring, fn, n, seed, extras):
    rng = np.random.default_rng(seed)
    buff = int(rng.choice([8 * 2048, 8 * 4096, 8 * 8192]))
    if extras and not ring.extras_available():
        pytest.skip("libnexr_extras.so not built (opt-in)")
    kinds = KINDS + (EXTRA_KINDS if extras else ())
    with ring.RingComm(n, ring.HOST_MEMORY, buff, fn, 30000, 0, None, None, 1 if n % 2 else 2, extras=extras) as comm:
        for step in range(40):
            kind = kinds[rng.integers(len(kinds))]
            count = int(rng.integers(1, 12_000))
            x = [rng.integers(0, 1 << 32, count * n, dtype=np.uint64).astype(np.uint32) for _ in range(n)]
            out = [np.full(count * n, 0xDEADBEEF, np.uint32) for _ in range(n)]
            total = np.zeros(count * n, np.uint64)
            for v in x:
                total += v
            total = (total & 0xFFFFFFFF).astype(np.uint32)
            root = int(rng.integers(n))
            what = (step, kind, count, root)
            if kind == "ar":
                comm.all_reduce(_ptrs(x), _ptrs(out), count, U32, 0)
                assert all(np.array_equal(o[:count], total[:count]) for o in out), what
            elif kind == "tree":
                comm.tree_all_reduce(_ptrs(x), _ptrs(out), count, U32, 0)
                assert all(np.array_equal(o[:count], total[:count]) for o in out), what
            elif kind == "rs":
                comm.reduce_scatter(_ptrs(x), _ptrs(out), count, U32, 0)
                for r in range(n):
                    assert np.array_equal(out[r][:count], total[r * count:(r + 1) * count]), what
            elif kind == "ag":
                comm.all_gather(_ptrs(x), _ptrs(out), count, U32)
                gathered = np.concatenate([v[:count] for v in x])
                assert all(np.array_equal(o, gathered) for o in out), what
            elif kind == "reduce":
                comm.reduce(_ptrs(x), _ptrs(out), count, U32, 0, root)
                assert np.array_equal(out[root][:count], total[:count]), what
            elif kind == "bcast":
                comm.broadcast(_ptrs(x), _ptrs(out), count, U32, root)
                assert all(np.array_equal(o[:count], x[root][:count]) for o in out), what
            else:
                shift = int(rng.integers(n))
                sp = [(r + shift) % n for r in range(n)]
                rp = [(r - shift) % n for r in range(n)]
                comm.send_recv(_ptrs(x), sp, _ptrs(out), rp, count * 4)
                for r in range(n):
                    assert np.array_equal(out[r][:count], x[rp[r]][:count]), what
