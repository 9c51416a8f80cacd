"""GPU parity tests of nexrReduceCopyBatch: every work of a batch against the oracle, bit-exact.

A batch carries many independent reduce-copies of one (datatype, op) — the analogue of one kernel
launch running a ncclDevWorkBatch (src/device/common.h:165-200) — so the cases mix K, M, sizes,
pointer phases and per-work op arguments (min next to max, different PreMulSum scalars and
divisors) inside one call, with more works than fit one launch, and check guard bytes around every
destination.
"""
import numpy as np
import pytest

import make_golden as mg
from test_reduce_copy_gpu import OPS, _case_args, _to_dev, same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


class _Work:
    def __init__(self, nexr, oracle, dt, op, name, k, m, n, seed, rng, offsets="random", in_place=False):
        esz = np.dtype(mg.STORE[dt]).itemsize
        if offsets == "zero":
            so, do = [0] * k, [0] * m
        elif offsets == "phase":
            ph = int(rng.integers(0, 16 // esz)) * esz
            so, do = [ph] * k, [ph] * m
        else:
            so = [int(rng.integers(0, 16)) for _ in range(k)]
            do = [int(rng.integers(0, 16)) for _ in range(m)]
        self.dt, self.n, self.esz, self.do = dt, n, esz, do
        self.arg, self.pre, self.post = _case_args(dt, name, op, k, rng)
        self.srcs = mg.gen_inputs(dt, k, max(n, 1), seed, special=True)
        if n == 0:
            self.srcs = [s[:0] for s in self.srcs]
        self.exp = oracle.reduce_copy(self.srcs, 1, dt, op, self.arg, self.pre, self.post)[0] if n else None
        self.sbufs = [_to_dev(s, o) for s, o in zip(self.srcs, so)]
        sptrs = [b.data_ptr() + o for b, o in zip(self.sbufs, so)]
        if in_place:
            self.dbufs, do = [self.sbufs[0]], [so[0]]
            self.do = do
            self.guard = False
        else:
            self.dbufs = [torch.full((n * esz + o + 64,), 0x5A, dtype=torch.uint8, device="cuda") for o in do]
            self.guard = True
        dptrs = [b.data_ptr() + o for b, o in zip(self.dbufs, do)]
        self.work = nexr.make_work(sptrs, dptrs, n, self.arg, self.pre, self.post)

    def check(self, tag):
        if self.n == 0:
            for b in self.dbufs:
                if self.guard:
                    assert (b.cpu().numpy() == 0x5A).all(), (tag, "empty work wrote")
            return
        for b, o in zip(self.dbufs, self.do):
            host = b.cpu().numpy()
            nb = self.n * self.esz
            if self.guard:
                assert (host[:o] == 0x5A).all() and (host[o + nb:] == 0x5A).all(), (tag, "write outside dst")
            got = host[o:o + nb].view(mg.STORE[self.dt])
            assert same(self.dt, got, self.exp), tag


SIZES = [0, 1, 2, 7, 15, 16, 17, 255, 1023, 4097, 65535, 300_001]


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES))
def test_batch_mixed_works_match_oracle(nexr, oracle, dt, dev):
    rng = np.random.default_rng(100 + dt)
    for name, op in OPS:
        if name == "sumpostdiv" and dt not in mg.INTS:
            continue
        n_works = int(rng.choice([1, 5, 14, 15, 37]))
        works = []
        for w in range(n_works):
            k = int(rng.integers(1, 9))
            m = int(rng.integers(1, 5))
            n = int(rng.choice(SIZES))
            mode = ["zero", "phase", "random"][int(rng.integers(0, 3))]
            works.append(_Work(nexr, oracle, dt, op, name, k, m, n, 9000 + 97 * w + op, rng, mode))
        nexr.reduce_copy_batch([w.work for w in works], dt, op, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for i, w in enumerate(works):
            w.check((mg.DT_NAMES[dt], name, i, w.n))


def test_batch_min_and_max_in_one_call(nexr, oracle, dev):
    # MinMax carries min/max in each work's redOpArg (reduce_kernel.h:64). The kernel is compiled per
    # isMin, so reduceCopyBatch runs a mixed batch as two launches, the min works and the
    # max works (nexr_api.cpp reduceCopyBatch); every work must still get its own op's result.
    rng = np.random.default_rng(7)
    for dt in (mg.I8, mg.U32, mg.F16, mg.F64):
        works = []
        for w in range(14):
            works.append(_Work(nexr, oracle, dt, mg.MINMAX, "max" if w % 2 else "min", 3, 1, 20_000 + w, 40 + w, rng))
        nexr.reduce_copy_batch([w.work for w in works], dt, mg.MINMAX)
        torch.cuda.synchronize()
        for i, w in enumerate(works):
            w.check((mg.DT_NAMES[dt], i))


def test_batch_in_place_and_large_works(nexr, oracle, dev):
    # Large works (tens of MiB) beside tiny ones: each gets its proportional workgroup range.
    rng = np.random.default_rng(11)
    works = [
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 2, 1, 8_000_003, 1, rng, "zero"),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 2, 2, 3, 2, rng, "random"),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 4, 1, 5_000_001, 3, rng, "phase", in_place=True),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 2, 1, 1, 4, rng, "zero", in_place=True),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 8, 3, 1_000_000, 5, rng, "random"),
    ]
    s = torch.cuda.Stream()
    nexr.reduce_copy_batch([w.work for w in works], mg.F32, mg.SUM, s.cuda_stream)
    s.synchronize()
    for i, w in enumerate(works):
        w.check(("large", i))


def test_batch_equals_separate_calls_bitwise(nexr, dev):
    # The same works through nexrReduceCopy one by one and through one batch give identical bytes.
    g = torch.Generator(device="cuda").manual_seed(3)
    srcs = [torch.randn(1 << 16, device="cuda", generator=g, dtype=torch.bfloat16) for _ in range(8)]
    works, outs_b, outs_s = [], [], []
    for i in range(1, 9):
        n = 1000 * i + i
        ob = torch.empty(n, device="cuda", dtype=torch.bfloat16)
        os_ = torch.empty_like(ob)
        ptrs = [t.data_ptr() + 2 * i for t in srcs[:i]]
        works.append(nexr.make_work(ptrs, [ob.data_ptr()], n))
        nexr.reduce_copy_ptrs(ptrs, [os_.data_ptr()], n, nexr.DataType.Bfloat16, nexr.DevRedOp.Sum,
                              stream=torch.cuda.current_stream().cuda_stream)
        outs_b.append(ob)
        outs_s.append(os_)
    nexr.reduce_copy_batch(works, nexr.DataType.Bfloat16, nexr.DevRedOp.Sum, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for a, b in zip(outs_b, outs_s):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("dt", [mg.F32, mg.BF16, mg.I8, mg.F64])
def test_multi_device_independent_chunks_match_oracle(nexr, oracle, dt, dev):
    """nexrReduceCopyMultiDevice (SURVEY §8(e), C5's independent chunks from one host call): every
    work on its own host thread and stream after a shared start barrier. On the one-GPU box every
    work names device 0 (several threads on one device); on a multi-GPU node work i takes GPU i mod n.
    Every work (all ops, mixed K/M/sizes/phases, reps > 1) against the oracle, guard bytes intact, the
    caller's current device unchanged."""
    rng = np.random.default_rng(500 + dt)
    n_dev = torch.cuda.device_count()
    for name, op in OPS:
        if name == "sumpostdiv" and dt not in mg.INTS:
            continue
        works = []
        for w in range(int(rng.choice([1, 3, 8]))):
            k, m = int(rng.integers(1, 9)), int(rng.integers(1, 3))
            n = int(rng.choice([0, 17, 4097, 300_001, 2_000_003]))
            d = w % n_dev
            with torch.cuda.device(d):
                works.append((_Work(nexr, oracle, dt, op, name, k, m, n, 7000 + 31 * w + op, rng,
                                    ["zero", "phase", "random"][w % 3]), d))
        torch.cuda.synchronize()
        before = torch.cuda.current_device()
        secs = nexr.reduce_copy_multi_device([w.work for w, _ in works], [d for _, d in works], dt, op,
                                             reps=int(rng.integers(1, 4)))
        assert torch.cuda.current_device() == before
        assert secs >= 0.0
        for i, (w, _) in enumerate(works):
            w.check((mg.DT_NAMES[dt], name, i, w.n))


@pytest.mark.parametrize("dt", [mg.F32, mg.BF16, mg.I8])
def test_multi_device_sets_rotate_and_match_oracle(nexr, oracle, dt, dev):
    """nexrReduceCopyMultiDeviceSets (the C5 fan-out's rotation): three sets of works per thread,
    launch k running set k mod 3; with reps = 4 every set runs at least once, and every set's output
    matches the oracle (mixed K, M, sizes and pointer phases across the sets); reps = 2 leaves the
    third set untouched (its guard-filled outputs unchanged), which shows the rotation order."""
    rng = np.random.default_rng(900 + dt)
    n_dev = torch.cuda.device_count()
    threads = 2
    per_dev = []
    for t in range(threads):
        with torch.cuda.device(t % n_dev):
            per_dev.append([_Work(nexr, oracle, dt, mg.SUM, "sum", int(rng.integers(1, 9)), int(rng.integers(1, 3)),
                                  int(rng.choice([17, 4097, 300_001])), 8000 + 10 * t + s, rng,
                                  ["zero", "phase", "random"][s]) for s in range(3)])
    torch.cuda.synchronize()
    devices = [t % n_dev for t in range(threads)]
    nexr.reduce_copy_multi_device_sets([[w.work for w in ws] for ws in per_dev], devices, dt, mg.SUM, reps=4)
    for t, ws in enumerate(per_dev):
        for s, w in enumerate(ws):
            w.check((mg.DT_NAMES[dt], "thread", t, "set", s))
    # reps = 2 on fresh outputs: sets 0 and 1 run, set 2 is never launched
    for ws in per_dev:
        for w in ws:
            for b in w.dbufs:
                b.fill_(0x5A)
    torch.cuda.synchronize()
    nexr.reduce_copy_multi_device_sets([[w.work for w in ws] for ws in per_dev], devices, dt, mg.SUM, reps=2)
    for t, ws in enumerate(per_dev):
        ws[0].check((mg.DT_NAMES[dt], "reps 2, thread", t, "set 0"))
        ws[1].check((mg.DT_NAMES[dt], "reps 2, thread", t, "set 1"))
        assert all((b.cpu().numpy() == 0x5A).all() for b in ws[2].dbufs), "set 2 ran with reps = 2"


def test_multi_device_rejects_bad_ordinals(nexr, dev):
    x = torch.ones(1024, device="cuda")
    y = torch.empty_like(x)
    work = nexr.make_work([x.data_ptr(), x.data_ptr()], [y.data_ptr()], 1024)
    for bad in (-1, torch.cuda.device_count()):
        with pytest.raises(nexr.NexrError) as e:
            nexr.reduce_copy_multi_device([work], [bad], mg.F32, 0)
        assert e.value.code == 4


def test_multi_device_concurrent_callers_share_the_stream_pool(nexr, dev):
    """Streams of nexrReduceCopyMultiDevice come from a process-wide per-device pool: four host
    threads calling it at once (two works each, several calls) never share a stream mid-call, every
    output is exact (integer-valued fp32, checked against torch on the device), and the pool stays
    bounded: a later burst of calls creates no new streams, so it costs no fresh-stream first-launch
    time."""
    import threading
    n = 1 << 20
    n_dev = torch.cuda.device_count()
    bufs = []
    for t in range(4):
        per = []
        for w in range(2):
            with torch.cuda.device((t + w) % n_dev):
                a = torch.randint(-1000, 1000, (n,), device="cuda").float()
                b = torch.randint(-1000, 1000, (n,), device="cuda").float()
                per.append((a, b, torch.empty_like(a), (t + w) % n_dev))
        bufs.append(per)
    torch.cuda.synchronize()
    errors = []

    def caller(t):
        try:
            per = bufs[t]
            works = [nexr.make_work([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n) for a, b, o, _ in per]
            for _ in range(6):
                nexr.reduce_copy_multi_device(works, [d for *_, d in per], mg.F32, 0, reps=2)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    created0, _ = nexr.pool_stats()
    threads = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
    [th.start() for th in threads]
    [th.join(timeout=60) for th in threads]
    assert not any(th.is_alive() for th in threads), "a caller thread hung (stream sharing or deadlock)"
    assert not errors, errors
    for per in bufs:
        for a, b, o, d in per:
            with torch.cuda.device(d):
                assert torch.equal(o, a + b)
    # The pool is bounded by the peak number of concurrent works (4 callers x 2 works), not by the
    # number of calls (4 x 6 calls x 2 works = 48).
    created1, _ = nexr.pool_stats()
    assert created1 - created0 <= 8, (created0, created1)
    # Warm pool: the same calls again, one thread after another, create no stream at all.
    for t in range(4):
        per = bufs[t]
        works = [nexr.make_work([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n) for a, b, o, _ in per]
        nexr.reduce_copy_multi_device(works, [d for *_, d in per], mg.F32, 0, reps=1)
    assert nexr.pool_stats()[0] == created1


def test_multi_device_c5_full_size_work_per_gpu(nexr, dev):
    """one full 256 MiB C2 work (fp32 sum, K=2, M=1) on EVERY visible GPU from one
    nexrReduceCopyMultiDevice call, each output checked bit-exactly on its own device (fp32 a+b is
    one IEEE add, so torch's a+b is the oracle's value). On the one-GPU box this is the N=1 case; on a
    node every GPU runs its own chunk at once."""
    n = 64 << 20
    n_dev = torch.cuda.device_count()
    works, devices, bufs = [], [], []
    for d in range(n_dev):
        with torch.cuda.device(d):
            g = torch.Generator(device=f"cuda:{d}")
            g.manual_seed(500 + d)
            a = torch.rand(n, device=f"cuda:{d}", generator=g) * 2 - 1
            b = torch.rand(n, device=f"cuda:{d}", generator=g) * 2 - 1
            o = torch.full_like(a, float("nan"))
            bufs.append((a, b, o))
            works.append(nexr.make_work([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n))
            devices.append(d)
    for d in range(n_dev):
        torch.cuda.synchronize(d)
    secs = nexr.reduce_copy_multi_device(works, devices, mg.F32, 0, reps=3)
    assert secs > 0
    for d, (a, b, o) in enumerate(bufs):
        with torch.cuda.device(d):
            assert torch.equal(o.view(torch.int32), (a + b).view(torch.int32)), f"GPU {d}"


def test_multi_device_c5_eight_chunks_folded_onto_one_call(nexr, dev):
    """C5's shape from one host call whatever the box: eight full 256 MiB C2 works (fp32 sum, K=2,
    M=1), work i on GPU i mod n. On the one-GPU box all eight threads share device 0, so the fan-out,
    its start barrier and eight concurrent one-shot grids on one device run at the node's work size
    (6 GiB of buffers); each output is checked bit-exactly (fp32 a+b is one IEEE add)."""
    n = 64 << 20
    n_dev = torch.cuda.device_count()
    works, devices, bufs = [], [], []
    for w in range(8):
        d = w % n_dev
        with torch.cuda.device(d):
            g = torch.Generator(device=f"cuda:{d}")
            g.manual_seed(700 + w)
            a = torch.rand(n, device=f"cuda:{d}", generator=g) * 2 - 1
            b = torch.rand(n, device=f"cuda:{d}", generator=g) * 2 - 1
            o = torch.full_like(a, float("nan"))
            bufs.append((a, b, o, d))
            works.append(nexr.make_work([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n))
            devices.append(d)
    for d in range(n_dev):
        torch.cuda.synchronize(d)
    secs = nexr.reduce_copy_multi_device(works, devices, mg.F32, 0, reps=2)
    assert secs > 0
    for w, (a, b, o, d) in enumerate(bufs):
        with torch.cuda.device(d):
            assert torch.equal(o.view(torch.int32), (a + b).view(torch.int32)), f"work {w} on GPU {d}"
    del bufs
    torch.cuda.empty_cache()


def test_batch_past_the_nt_store_threshold_runs_single_launches(nexr, oracle, dev):
    """Round 6: batch kernels are compiled for the plain and nt-load policies only; a run of works that
    streams >= 512 MiB (where a single launch would take nt stores) is launched work by work, each at
    its own policy. Two 104 MiB works and a small one of the same (datatype, op, K): 632 MiB streamed,
    all exact, with a K = 1 copy and a signed-integer Sum batch beside them (routed kernels)."""
    rng = np.random.default_rng(31)
    works = [
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 2, 1, 26 << 20, 1, rng, "zero"),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 2, 1, 5_000, 2, rng, "phase"),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 2, 1, 26 << 20, 3, rng, "random"),
        _Work(nexr, oracle, mg.F32, mg.SUM, "sum", 1, 2, 1_000_003, 4, rng, "phase"),
    ]
    nexr.reduce_copy_batch([w.work for w in works], mg.F32, mg.SUM)
    torch.cuda.synchronize()
    for i, w in enumerate(works):
        w.check(("nt-store run", i))
    del works
    torch.cuda.empty_cache()
    for op, name in ((mg.SUM, "sum"), (mg.PROD, "prod")):
        sub = [_Work(nexr, oracle, mg.I32, op, name, k, 1, 70_001 + k, 10 + k, rng, "random") for k in (1, 2, 3)]
        nexr.reduce_copy_batch([w.work for w in sub], mg.I32, op)
        torch.cuda.synchronize()
        for i, w in enumerate(sub):
            w.check(("int32 routed", name, i))
