"""The xGMI peer-step probe (tools/xgmi_probe.py). Only the driver's 8-GPU node can
run its measurement; here the probe must report "skipped" cleanly, and bench.py's wrapper must turn
any failure of the probe into a reported field instead of an exception."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_probe_skips_without_two_gpus():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs present: the probe measures instead of skipping")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "xgmi_probe.py")], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    assert "skipped" in json.loads(line)


def test_bench_wrapper_reports_failures(monkeypatch):
    import bench
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)  # the probe's parts run only with 2+ GPUs

    class Boom:
        pid = 999_999_999
        returncode = 3

        def __init__(self, *a, **k):
            pass

        def communicate(self, timeout=None):
            return "", "boom"

    monkeypatch.setattr(subprocess, "Popen", Boom)
    r = bench.xgmi_probe()
    assert r["error"] == "exit 3" and "boom" in r["stderr"]

    killed = []

    class Hang(Boom):
        calls = 0

        def communicate(self, timeout=None):
            Hang.calls += 1
            if Hang.calls == 1:
                raise subprocess.TimeoutExpired("x", 1)
            return "", ""

    monkeypatch.setattr(subprocess, "Popen", Hang)
    monkeypatch.setattr(os, "killpg", lambda pid, sig: killed.append(pid))
    assert "timeout" in bench.xgmi_probe()["error"]
    assert killed == [Hang.pid]  # the probe's whole process group, not just the probe
