"""CPU tests of bench.py's JSON lines (no GPU): the launcher-free N>1 fan-out (one process driving N
GPUs through nexrReduceCopyMultiDevice) with a faked device count and faked timings, the C5 summary
arithmetic, and the CPU-baseline core count. The GPU measurement itself runs on the MI355X box."""
import argparse
import json
import types

import pytest

import bench


class _FakeWorkload:
    made = []

    def __init__(self, pkg, cfg, device_index, seed, sets=3):
        self.device_index = device_index
        _FakeWorkload.made.append(device_index)

    def work(self, i=0):
        return ("work", self.device_index)

    def run(self, steps, warmup, dist, per_launch=False):
        return 0.0, 0.0, 125e-6  # 125 us per launch

    def free(self):
        pass


class _FakePkg:
    def __init__(self):
        self.calls = []

    def reduce_copy_multi_device(self, works, devices, dt, op, reps=1):
        self.calls.append((list(devices), reps))
        # 0.125 ms per step per GPU alone; 2 % slower with every GPU busy
        per = 0.125e-3 * (1.02 if len(devices) > 1 else 1.0)
        return per * reps * (1 + 0.001 * devices[0])


def _args(**kw):
    a = dict(gpus=4, steps=20, warmup=5, config="c2", cpu_seconds=1.0, no_cpu=True, no_h2d=True, no_extra=True,
             no_xgmi=True, events="region")
    a.update(kw)
    return argparse.Namespace(**a)


def test_fanout_line_shape(monkeypatch, capsys):
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 4)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(bench, "DeviceWorkload", _FakeWorkload)
    _FakeWorkload.made = []
    pkg = _FakePkg()
    cfg = bench.CONFIGS["c2"]
    res = bench.main_fanout(_args(), cfg, pkg)
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line == json.loads(json.dumps(res))
    # driver contract keys
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config"):
        assert key in line, key
    assert line["n_gpus"] == 4 and line["steps"] == 20 and line["warmup"] == 5 and line["scaling"] == "weak"
    assert line["metric"] == bench.METRIC and line["dtype"] == "f32"
    bytes_step = bench.algorithmic_bytes(cfg)
    agg_s = 0.125e-3 * 1.02 * 20
    assert line["value"] == pytest.approx(4 * bytes_step * 20 / agg_s / 1e9, rel=1e-4)
    assert line["ms_per_step"] == pytest.approx(agg_s / 20 * 1e3, abs=1e-4)
    # all four GPUs together, then each alone, each with W untimed reps first
    assert pkg.calls[0] == ([0, 1, 2, 3], 5) and pkg.calls[1] == ([0, 1, 2, 3], 20)
    assert [c for c in pkg.calls[2:]] == [([d], r) for d in range(4) for r in (5, 20)]
    c5 = line["c5"]
    assert c5["n1_same_run_gbs"] == pytest.approx(bytes_step * 20 / (0.125e-3 * 20) / 1e9, rel=1e-3)
    assert len(c5["solo_gbs_per_gpu"]) == 4
    assert c5["aggregate_over_n_times_n1"] == pytest.approx(1 / 1.02, rel=1e-3)
    assert line["roofline"]["avg_kernel_us"] == 125.0
    assert line["roofline"]["frac"] == pytest.approx(bytes_step / 125e-6 / 1e9 / 8000, abs=1e-4)
    assert "nexrReduceCopyMultiDevice" in line["config"]["parallelism"]


def test_fanout_refuses_more_gpus_than_visible(monkeypatch):
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(SystemExit):
        bench.main_fanout(_args(gpus=2), bench.CONFIGS["c2"], _FakePkg())


def test_fanout_rehearsal_folds_chunks_onto_visible_gpus(monkeypatch, capsys):
    """NEXR_BENCH_FOLD=1: 2 chunks on a 1-GPU box both run on GPU 0 and the line says REHEARSAL."""
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(bench, "DeviceWorkload", _FakeWorkload)
    monkeypatch.setenv("NEXR_BENCH_FOLD", "1")
    _FakeWorkload.made = []
    pkg = _FakePkg()
    bench.main_fanout(_args(gpus=2), bench.CONFIGS["c2"], pkg)
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert pkg.calls[0] == ([0, 0], 5) and pkg.calls[2:] == [([0], 5), ([0], 20)] * 2
    assert "REHEARSAL: 2 chunks folded onto 1 GPU(s)" in line["config"]["parallelism"]
    assert line["n_gpus"] == 2


def test_c5_summary_arithmetic():
    s = bench.c5_summary(8, 1 << 30, 10, agg_seconds=0.02, n1_seconds=0.016, solo_seconds=[0.016] * 8)
    assert s["aggregate_gbs"] == round(8 * (1 << 30) * 10 / 0.02 / 1e9, 2)
    assert s["n1_same_run_gbs"] == round((1 << 30) * 10 / 0.016 / 1e9, 2)
    assert s["aggregate_over_n_times_n1"] == pytest.approx(0.8)


def test_usable_cores_is_affinity_capped_by_quota(monkeypatch, tmp_path):
    import builtins
    import os
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(128)))
    real_open = builtins.open

    def fake_open(path, *a, **k):
        if path == "/sys/fs/cgroup/cpu.max":
            p = tmp_path / "cpu.max"
            p.write_text("1600000 100000\n")
            return real_open(p, *a, **k)
        return real_open(path, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)
    n, how = bench.usable_cores()
    assert n == 16 and "128" in how and "16" in how


def test_cpu_baseline_runs_the_full_configuration(monkeypatch):
    """The CPU baseline times the benchmarked call itself: every buffer at the config's size."""
    seen = {}
    import oracle

    def fake_rc(srcs, m, dt, op, arg, dsts=None, threads=1, emulated=None):
        seen.setdefault("n", srcs[0].size)
        seen.setdefault("first", (threads, emulated))
        seen.setdefault("modes", set()).add((threads > 1, emulated))
        seen["threads"] = threads
        return dsts

    monkeypatch.setattr(oracle, "reduce_copy", fake_rc)
    cfg = dict(bench.CONFIGS["c4_i8_min"])
    cfg["buf_bytes"] = 1 << 20  # keep the sample small here; the shape is what is checked
    e = bench.cpu_baseline_entry(cfg, seconds=0.05)
    assert seen["n"] == 1 << 20
    assert e["cores"] == 1 and e["kind"] == "port" and "1 MiB" in e["sample"]
    assert e["all_cores"]["cores"] == bench.usable_cores()[0] == seen["threads"]
    assert "1.79" in e["note"]
    # the headline is the reference's execution (480 emulated threads, Unroll 4) on one core; the
    # plain element loop is reported beside it, both on 1 and on all cores
    assert seen["first"] == (1, (480, 4))
    assert seen["modes"] == {(False, (480, 4)), (True, (480, 4)), (False, None), (True, None)}
    assert e["element_loop"]["cores"] == 1 and e["element_loop"]["all_cores"] == bench.usable_cores()[0]


def test_bounded_probe_kills_its_whole_process_group(tmp_path):
    """bench._bounded (the xGMI probes after the timed region): a probe that hangs is killed together
    with the ring ranks it started, and the line records the timeout instead of failing."""
    import subprocess
    import sys
    import time
    pidfile = tmp_path / "grandchild.pid"
    script = tmp_path / "hang.py"
    script.write_text(
        "import subprocess, sys, time\n"
        f"g = subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(600)'])\n"
        f"open({str(pidfile)!r}, 'w').write(str(g.pid))\n"
        "time.sleep(600)\n")
    t0 = time.time()
    res = bench._bounded([sys.executable, str(script)], 3.0)
    assert "timeout" in res["error"] and time.time() - t0 < 30
    gpid = int(pidfile.read_text())
    for _ in range(50):
        if subprocess.run(["kill", "-0", str(gpid)], capture_output=True).returncode != 0:
            break
        time.sleep(0.1)
    else:
        raise AssertionError("the probe's child survived the timeout")
    ok = bench._bounded([sys.executable, "-c", "print('{\"a\": 1}')"], 30.0)
    assert ok == {"a": 1}
    bad = bench._bounded([sys.executable, "-c", "import sys; sys.exit(3)"], 30.0)
    assert bad["error"] == "exit 3"


def test_side_leg_records_failures():
    """A failing leg after the headline's timed region lands in the line as an error, not a crash."""
    import bench

    def c1_ring():
        raise RuntimeError("peer access refused")

    r = bench.side_leg(c1_ring)
    assert r["leg"] == "c1_ring" and "peer access refused" in r["error"]
    assert bench.side_leg(lambda a, b: a + b, 2, 3) == 5
