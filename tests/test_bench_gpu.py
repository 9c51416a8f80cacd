"""bench.py end to end on the GPU, each run in a fresh interpreter exactly as the driver starts it
(round 2 began with a bench that failed at its first launch while every other GPU test passed: the
library was loaded before torch and two HIP runtimes were mapped). Short runs; the line must carry the
driver's keys and the measurement blocks, and every rate must be positive and below the HBM peak."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline")


def _line(cmd, env=None, timeout=240):
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stdout[-1500:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"stdout must be exactly one JSON line, got {len(lines)}: {p.stdout[-800:]}"
    d = json.loads(lines[0])
    for k in KEYS:
        assert k in d, k
    assert 0 < d["value"] and 0 < d["roofline"]["achieved"] < d["roofline"]["peak"]
    return d


def test_bench_default_line_short():
    d = _line([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-h2d", "--no-extra"])
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["config"]["k_inputs"] == 2


def test_bench_extra_configs_and_c1():
    d = _line([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-h2d"])
    assert set(d["extra_configs"]) == {"c3_f16", "c3_bf16", "c4_i32_min", "c4_i32_max", "c4_i32_prod", "c4_i8_min",
                                       "c4_i8_max", "c4_i8_prod"}
    for v in d["extra_configs"].values():
        assert 0 < v["frac"] < 1
    assert "error" not in d["c1_ring"], d["c1_ring"]
    assert all(d["c1_ring"][k]["exact"] for k in ("device", "device_ll", "device_ll128", "host_staged", "cpu_oracle"))
    assert d["c1_ring"]["device"]["step_wait"] == "word"  # both emulated ranks on the one GPU
    assert "resident_ring" not in d and "device_resident" not in d["c1_ring"]  # extras: not in the default line


def test_bench_fanout_rehearsal():
    d = _line([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-xgmi"],
              env={"NEXR_BENCH_FOLD": "1"})
    assert d["n_gpus"] == 2 and "c5" in d
    assert d["phase_s"]["total"] < d["phase_s"]["cap_s"]


def test_bench_torchrun_two_ranks():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    d = _line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
               "--no-xgmi"])
    assert d["n_gpus"] == 2 and len(d["per_gpu"]["wall_gbs"]) == 2 and "c5" in d
