"""World-size-2 rehearsal of bench.py's N>1 path on CPU (gloo): every rank processes its own
independent chunk (no data-path collective), the timed region is bracketed by
barriers, and the reported time is the MAX over ranks. The per-rank step here is the CPU oracle
standing in for the device launch (the GPU step itself is covered by tests -m gpu)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import time
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests", "golden")]
    import bench
    import make_golden as mg
    import oracle

    d = bench.Dist("gloo")
    srcs = mg.gen_inputs(mg.F32, 2, 50_000, 1000 + rank * 7, special=False)  # rank-own chunk
    out = [None]

    def step(i):
        if rank == 1:
            time.sleep(0.01)  # skew: rank 1 is the slow one
        out[0] = oracle.reduce_copy(srcs, 1, mg.F32, mg.SUM)[0]

    local, mx = bench.timed_steps(step, steps=5, warmup=1, sync=lambda: None, dist=d)
    ok = np.array_equal(out[0], (srcs[0] + srcs[1]).astype(np.float32))
    gathered = d.gather([local, float(rank)])
    summary = bench.per_gpu_summary(gathered, bytes_step=1 << 20, steps=5)
    d.close()
    q.put((rank, local, mx, ok, gathered, summary))


def test_two_rank_independent_chunks_max_timer():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    assert all(p.exitcode == 0 for p in ps)
    (r0, l0, m0, ok0, g0, s0), (r1, l1, m1, ok1, g1, s1) = res
    assert ok0 and ok1
    assert m0 == m1 == max(l0, l1)
    assert l1 >= 0.05  # the skewed rank's 5 steps
    # per-rank breakdown of the N > 1 bench line: every rank sees every rank's time, in rank order
    assert g0 == g1 == [[l0, 0.0], [l1, 1.0]]
    assert s0 == s1 and len(s0["wall_gbs"]) == 2
    assert s0["min_wall_gbs"] == round(5 * (1 << 20) / l1 / 1e9, 2)  # the slow rank sets the minimum


def test_rank_stdout_is_only_the_json_line(tmp_path):
    """gloo's native "[Gloo] Rank r is connected to ..." lines go to fd 1; bench.Dist routes them to
    stderr so that rank 0's stdout under torchrun is exactly the driver's one JSON line."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "rank.py"
    script.write_text(f"import sys; sys.path.insert(0, {root!r}); import bench\n"
                      "d = bench.Dist('gloo'); print('{\"rank\": %d}' % d.rank); d.close()\n")
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert [o for o, _ in outs] == ['{"rank": 0}\n', '{"rank": 1}\n']


def _h2d_rank_main(rank, world, port, q, fail_rank):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    import bench
    import torch

    class FakePkg:  # stands in for the library: "copies" host buffers, or fails on one rank
        def reduce_copy_ptrs(self, *a, **k):
            if rank == fail_rank:
                raise RuntimeError("pinning failed on this rank")

    # torch pin_memory needs a GPU runtime; on CPU stand it in with the plain tensor
    torch.Tensor.pin_memory = lambda self: self
    d = bench.Dist("gloo")
    cfg = dict(bench.CONFIGS["c2"])
    cfg["buf_bytes"] = 1 << 20
    res = bench.h2d_pinned_all_ranks(FakePkg(), cfg, d, None, reps=2)
    d.close()
    q.put((rank, res))


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_node_wide_h2d_leg_survives_a_failing_rank(fail_rank):
    """bench.py's N > 1 host-inclusive leg: every rank joins the barrier and the gather even when one
    rank fails, and the line records the failure instead of hanging or raising."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_h2d_rank_main, args=(r, 2, port, q, fail_rank)) for r in range(2)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    assert all(p.exitcode == 0 for p in ps)
    if fail_rank < 0:
        assert res[0]["value"] > 0 and len(res[0]["per_rank_gbs"]) == 2
    else:
        assert "error" in res[0] and "error" in res[1]
        assert "pinning failed" in res[1]["error"]
