"""Random sequences of every emulated collective on ONE device-memory communicator with the MI355X
kernels underneath (the GPU twin of test_mixed_sequences.py): links, FIFOs in HBM and step
counters shared across ring, tree, PAT and send/recv calls. Integer sums: exact expected values."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

U32 = 3
KINDS = ("ar", "rs", "ag", "reduce", "bcast", "tree")
EXTRA_KINDS = ("sendrecv",)  # the opt-in extras library (include/nexr_extras.h)


@pytest.fixture(scope="module")
def ring(nexr):
    assert torch.cuda.is_available()
    return importlib.import_module("nex-nccl_amd.ring")


@pytest.mark.parametrize("n,seed", [(2, 21), (3, 22), (4, 23), (8, 24)])
@pytest.mark.parametrize("extras", [False, True])
def test_random_collective_sequences_device(ring, n, seed, extras):
    rng = np.random.default_rng(seed)
    buff = int(rng.choice([8 * 4096, 8 * 16384, 1 << 20]))
    if extras and not ring.extras_available():
        pytest.skip("libnexr_extras.so not built (opt-in)")
    kinds = KINDS + (EXTRA_KINDS if extras else ())
    with ring.RingComm(n, ring.DEVICE_MEMORY, buff, tree_ranks_per_node=1 if n % 2 else 2, extras=extras) as comm:
        for step in range(30):
            kind = kinds[rng.integers(len(kinds))]
            count = int(rng.integers(1, 200_000))
            xs = [rng.integers(0, 1 << 32, count * n, dtype=np.uint64).astype(np.uint32) for _ in range(n)]
            total = np.zeros(count * n, np.uint64)
            for v in xs:
                total += v
            total = (total & 0xFFFFFFFF).astype(np.uint32)
            x = [torch.from_numpy(v.view(np.int32)).cuda() for v in xs]
            out = [torch.full((count * n,), -1, dtype=torch.int32, device="cuda") for _ in range(n)]
            torch.cuda.synchronize()
            xp, op = [t.data_ptr() for t in x], [t.data_ptr() for t in out]
            root = int(rng.integers(n))
            what = (step, kind, count, root)
            got = lambda r: out[r].cpu().numpy().view(np.uint32)  # noqa: E731
            if kind in ("ar", "tree"):
                (comm.all_reduce if kind == "ar" else comm.tree_all_reduce)(xp, op, count, U32, 0)
                assert all(np.array_equal(got(r)[:count], total[:count]) for r in range(n)), what
            elif kind == "rs":
                comm.reduce_scatter(xp, op, count, U32, 0)
                for r in range(n):
                    assert np.array_equal(got(r)[:count], total[r * count:(r + 1) * count]), what
            elif kind == "ag":
                comm.all_gather(xp, op, count, U32)
                gathered = np.concatenate([v[:count] for v in xs])
                assert all(np.array_equal(got(r), gathered) for r in range(n)), what
            elif kind == "reduce":
                comm.reduce(xp, op, count, U32, 0, root)
                assert np.array_equal(got(root)[:count], total[:count]), what
            elif kind == "bcast":
                comm.broadcast(xp, op, count, U32, root)
                assert all(np.array_equal(got(r)[:count], xs[root][:count]) for r in range(n)), what
            else:
                shift = int(rng.integers(n))
                sp = [(r + shift) % n for r in range(n)]
                rp = [(r - shift) % n for r in range(n)]
                comm.send_recv(xp, sp, op, rp, count * 4)
                for r in range(n):
                    assert np.array_equal(got(r)[:count], xs[rp[r]][:count]), what
