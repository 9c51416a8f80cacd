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
        self.dev = None
        _FakeWorkload.made.append(device_index)

    def work(self, i=0):
        return ("work", self.device_index, i)

    def run(self, steps, warmup, dist, per_launch=False):
        self.last_set = (steps + warmup - 1) % 3
        return 2.5e-3, 2.5e-3, 125e-6  # 125 us per launch

    def per_set(self, rounds=6):
        return {"per_set_us": [125.0, 124.0, 126.0], "per_set_frac": [0.8, 0.81, 0.79], "per_set_launches": rounds,
                "per_set_buffers_mib": [[0.0, 256.0, 512.0]] * 3}

    def check_exact(self, i):
        return {"exact": True, "checked_elements": 1 << 20, "checked_set": i}

    def free(self):
        pass


class _FakePkg:
    def __init__(self):
        self.calls = []

    def reduce_copy_multi_device_sets(self, works, devices, dt, op, reps=1):
        # three rotating sets on every GPU, each GPU's own
        assert all(len(w) == 3 and [x[2] for x in w] == [0, 1, 2] for w in works)
        assert [w[0][1] for w in works] == list(devices)
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
    assert "nexrReduceCopyMultiDeviceSets" in line["config"]["parallelism"]
    assert line["c5"]["sets_per_gpu"] == 3 and "3 rotating" in line["config"]["parallelism"]
    assert _FakeWorkload.made == [0, 1, 2, 3, 0]  # one 3-set workload per GPU, then GPU 0's roofline leg
    assert line["exact"] is True and line["exact_check"]["per_gpu"] == [True] * 4
    assert line["roofline"]["per_set_us"] == [125.0, 124.0, 126.0]


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


def test_n1_line_carries_exact_and_per_set(monkeypatch, capsys):
    """The N=1 line: `exact` (bit-exact check of the last launch's output vs the oracle, outside the
    timed region) and `roofline.per_set_us` for the headline, and the same keys for every one of
    the eight extra configurations (a skipped GPUTEST must not leave the bench's work
    unproven)."""
    import torch
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a, **k: None)
    monkeypatch.setattr(bench, "DeviceWorkload", _FakeWorkload)
    monkeypatch.setattr(bench, "c1_ring", lambda: {"skipped": "test"})
    res = bench.main_ranks(_args(gpus=1, no_extra=False), bench.CONFIGS["c2"], _FakePkg())
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line == json.loads(json.dumps(res))
    assert line["exact"] is True and line["exact_check"]["checked_elements"] >= 1 << 20
    assert line["roofline"]["per_set_us"] == [125.0, 124.0, 126.0] and len(line["roofline"]["per_set_buffers_mib"]) == 3
    extra = line["extra_configs"]
    assert sorted(extra) == sorted(bench.EXTRA_ORDER)
    for name, e in extra.items():
        assert e["exact"] is True and len(e["per_set_us"]) == 3 and len(e["per_set_frac"]) == 3, name


@pytest.mark.parametrize("name", ["c2", "c3_bf16", "c4_i8_min", "c4_i32_prod"])
def test_check_exact_against_the_oracle_on_cpu_tensors(name):
    """DeviceWorkload.check_exact itself (CPU tensors standing in for HBM): the output the oracle
    gives passes, a one-bit flip anywhere in the sample fails, and the sample covers >= 1 Mi elements
    spread over the buffer including its first and last run."""
    import numpy as np
    import torch
    import oracle
    cfg = dict(bench.CONFIGS[name])
    cfg["buf_bytes"] = 8 << 20 if name != "c4_i8_min" else 4 << 20
    esz = bench.ESZ[cfg["dt"]]
    n = cfg["buf_bytes"] // esz
    rng = np.random.default_rng(0)
    srcs = [torch.from_numpy(rng.integers(0, 256, cfg["buf_bytes"], dtype=np.uint8)) for _ in range(cfg["k"])]
    if cfg["dt"] in (6, 7, 9):  # finite floats, as the bench's uniform data
        fl = {6: torch.float16, 7: torch.float32, 9: torch.bfloat16}[cfg["dt"]]
        srcs = [(torch.rand(n, generator=torch.Generator().manual_seed(i)) * 2 - 1).to(fl) for i in range(cfg["k"])]
    exp = oracle.reduce_copy([s.view(torch.uint8).numpy() for s in srcs], 1, cfg["dt"], cfg["op"], cfg["arg"])[0]
    dst = torch.from_numpy(exp.view(np.uint8).copy())
    wl = object.__new__(bench.DeviceWorkload)
    wl.cfg, wl.n, wl.dev = cfg, n, torch.device("cpu")
    wl.sets = [([0] * cfg["k"], [0], srcs, [dst])]
    r = wl.check_exact(0)
    assert r["exact"] is True and r["checked_elements"] >= 1 << 20 or r["checked_elements"] == n
    for pos in (0, n // 2, n - 1):  # first run, a run in the middle (if sampled), last run
        bad = dst.clone()
        bad.view(torch.uint8)[pos * esz] ^= 1
        wl.sets = [([0] * cfg["k"], [0], srcs, [bad])]
        r2 = wl.check_exact(0, blocks=256, block=64)
        starts = set(int(x) for x in np.linspace(0, n - 64, 256)) | {0, n - 64}
        sampled = any(s <= pos < s + 64 for s in starts)
        assert r2["exact"] is (not sampled), pos


def _ring_result(cmd, exact=True, gpus=(0, 1)):
    wait = cmd[cmd.index("--step-wait") + 1] if "--step-wait" in cmd else "default"
    return {"gpus": list(gpus), "exact_all_ranks": exact, "step_wait": wait, "step_wait_in_effect": [wait],
            "per_protocol_bytes": {"simple": {"4194304": {"ms": 0.1, "algbw_GBps": 41.9, "exact": exact}}}}


def test_xgmi_probe_parts_link_rates_and_timeouts(monkeypatch, capsys):
    """N>1 with the xGMI probe on (faked: 4 GPUs, faked probe outputs): every part runs in its own
    bounded subprocess; the remote read/write and every ring result carry their rate against the
    153 GB/s one-link bound next to their exact check; both process rings run under both step waits
    (sync first, then the completion word) and the line carries both; a part that times out is
    recorded as such and the headline line is still printed, with its phase times."""
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 4)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(bench, "DeviceWorkload", _FakeWorkload)
    seen = []

    def fake_bounded(cmd, timeout_s):
        arg = cmd[2]
        wait = cmd[cmd.index("--step-wait") + 1] if "--step-wait" in cmd else None
        seen.append((arg, wait, timeout_s))
        if arg == "--peer-step":
            return {"gpus": [0, 1], "remote_read": {"xgmi_GBps": 76.5, "exact": True},
                    "remote_write": {"xgmi_GBps": 122.4, "exact": True}}
        if arg == "--ring-only":
            return _ring_result(cmd)
        if arg == "--resident-only":
            return {"ranks": 4, "ch1_4194304": {"ms": 0.2, "algbw_GBps": 20.0, "busbw_GBps": 30.0, "exact": True}}
        return {"error": f"timeout after {timeout_s:.0f} s"}  # --ring-all hangs

    monkeypatch.setattr(bench, "_bounded", fake_bounded)
    monkeypatch.setenv("NEXR_XGMI_RESIDENT", "1")
    bench.main_fanout(_args(no_xgmi=False), bench.CONFIGS["c2"], _FakePkg())
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["n_gpus"] == 4 and line["value"] > 0  # the headline is there
    x = line["xgmi_probe"]
    assert [(a, w) for a, w, _ in seen] == [("--peer-step", None), ("--ring-only", "sync"), ("--ring-only", "word"),
                                            ("--ring-all", "sync"), ("--ring-all", "word"), ("--resident-only", None)]
    assert all(t <= 60 for _, _, t in seen)
    assert x["link_bound_GBps"] == 153.0
    assert x["remote_read"]["frac_of_link"] == pytest.approx(76.5 / 153, abs=1e-4)
    assert x["remote_write"]["frac_of_link"] == pytest.approx(122.4 / 153, abs=1e-4)
    for key in ("ring_processes", "ring_processes_word"):
        r = x[key]["per_protocol_bytes"]["simple"]["4194304"]
        assert r["busbw_GBps"] == pytest.approx(41.9, abs=0.01) and r["frac_of_link"] == pytest.approx(41.9 / 153, abs=1e-3)
    assert x["ring_processes"]["step_wait"] == "sync" and x["ring_processes_word"]["step_wait"] == "word"
    modes = x["step_wait_modes"]
    assert modes["ring_processes"]["sync_exact_all_ranks"] is True and modes["ring_processes"]["word_exact_all_ranks"] is True
    assert modes["visibility_fault"] is False and modes["link_or_schedule_fault"] is False
    assert x["resident_ring"]["ch1_4194304"]["frac_of_link"] == pytest.approx(30 / 153, abs=1e-3)
    assert "timeout" in x["ring_processes_all_gpus"]["error"] and "timeout" in x["ring_processes_all_gpus_word"]["error"]
    assert set(x["part_s"]) == {"peer_step", "ring_processes", "ring_processes_word", "ring_processes_all_gpus",
                                "ring_processes_all_gpus_word", "resident_ring"}
    ph = line["phase_s"]
    for k in ("startup", "inputs", "timed_region", "solo_legs", "exact_checks", "xgmi_probe", "total"):
        assert k in ph, k
    assert ph["cap_s"] == bench.TOTAL_CAP_S


@pytest.mark.parametrize("word_exact,sync_exact,visibility,link", [(False, True, True, False), (True, False, False, True),
                                                                    (False, False, False, True)])
def test_step_wait_verdict_tells_visibility_from_link_faults(monkeypatch, word_exact, sync_exact, visibility, link):
    """The first multi-GPU line must tell a step-visibility fault (the completion word wrong, the
    synchronisation right) from a link or schedule fault (the synchronisation wrong too)."""
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("NEXR_XGMI_RESIDENT", raising=False)

    def fake_bounded(cmd, timeout_s):
        if cmd[2] == "--peer-step":
            return {"gpus": [0, 1]}
        wait = cmd[cmd.index("--step-wait") + 1]
        return _ring_result(cmd, exact=word_exact if wait == "word" else sync_exact,
                            gpus=range(8) if cmd[2] == "--ring-all" else (0, 1))

    monkeypatch.setattr(bench, "_bounded", fake_bounded)
    res = bench.xgmi_probe()
    m = res["step_wait_modes"]
    assert m["visibility_fault"] is visibility and m["link_or_schedule_fault"] is link
    assert m["ring_processes_all_gpus"]["word_exact_all_ranks"] is word_exact
    assert m["ring_processes_all_gpus"]["sync_in_effect"] == ["sync"]


def test_probe_budget_caps_the_line():
    """The N > 1 line stays under TOTAL_CAP_S (300 s; the driver's BENCH timeout is 600 s): the probe
    gets at most XGMI_BUDGET_S and never more than what the earlier phases left."""
    assert bench.TOTAL_CAP_S <= 300 and bench.XGMI_BUDGET_S <= bench.TOTAL_CAP_S
    assert bench.probe_budget(0.0) == bench.XGMI_BUDGET_S
    assert bench.probe_budget(200.0) == pytest.approx(bench.TOTAL_CAP_S - bench.XGMI_MARGIN_S - 200.0)
    assert bench.probe_budget(bench.TOTAL_CAP_S) == 0.0
    for elapsed in (0.0, 60.0, 150.0, 280.0):
        assert elapsed + bench.probe_budget(elapsed) <= bench.TOTAL_CAP_S


def test_probe_parts_share_the_budget(monkeypatch):
    """Every part that hangs is charged its whole limit (a faked clock): the parts together never
    take more than the budget, and the ones that find it spent are recorded, not run."""
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("NEXR_XGMI_RESIDENT", raising=False)
    clock = [1000.0]
    monkeypatch.setattr(bench.time, "perf_counter", lambda: clock[0])
    granted = []

    def hang(cmd, timeout_s):
        granted.append(timeout_s)
        clock[0] += timeout_s
        return {"gpus": [0, 1]} if cmd[2] == "--peer-step" else {"error": f"timeout after {timeout_s:.0f} s"}

    monkeypatch.setattr(bench, "_bounded", hang)
    budget = 120.0
    res = bench.xgmi_probe(budget)
    assert sum(granted) <= budget + 1e-6
    assert res["wall_s"] <= budget
    spent = [k for k in ("ring_processes_all_gpus", "ring_processes_all_gpus_word")
             if "budget is spent" in res.get(k, {}).get("error", "")]
    assert spent  # 45 + 40 + 40 = 125 > 120: the later parts were skipped


def test_xgmi_probe_resident_parts_opt_in(monkeypatch):
    """Without NEXR_XGMI_RESIDENT=1 the probe runs only row f4's parts (the peer step and the
    host-sequenced process rings); the device-resident ring (extras library) is not launched."""
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("NEXR_XGMI_RESIDENT", raising=False)
    seen = []
    monkeypatch.setattr(bench, "_bounded", lambda cmd, t: seen.append(cmd[2]) or {"gpus": [0, 1]})
    res = bench.xgmi_probe()
    assert seen == ["--peer-step", "--ring-only", "--ring-only", "--ring-all", "--ring-all"]
    assert "resident_ring" not in res


def test_xgmi_probe_skipped_on_one_gpu(monkeypatch):
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    calls = []
    monkeypatch.setattr(bench, "_bounded", lambda cmd, t: calls.append(cmd) or {})
    res = bench.xgmi_probe()
    assert "skipped" in res and calls == []


def test_comparator_sequence_orders():
    """The per-set comparator (DeviceWorkload.per_set): both orders launch the kernel and the uint32 sum
    `rounds` times on every set; "grouped" never launches on the set the previous launch used (so
    neither side finds the other's bytes in the Infinity Cache), "paired" does so by construction."""
    for ns in (2, 3, 4):
        for order in ("grouped", "paired"):
            seq = bench.comparator_sequence(ns, 5, order)
            assert sorted(seq) == sorted((kd, j) for kd in (0, 1) for j in range(ns) for _ in range(5))
            same = sum(a[1] == b[1] for a, b in zip(seq, seq[1:]))
            assert (same == 0) if order == "grouped" else (same == 5 * ns)
    with pytest.raises(ValueError):
        bench.comparator_sequence(3, 1, "other")
