"""CPU checks of the committed HBM-traffic summaries (profiles/pmc_<config>.json) that bench.py puts
in `roofline.traffic`, and of the tool that makes them (tools/pmc_traffic.py)."""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_every_config_has_a_plausible_traffic_summary():
    import bench
    for name in bench.CONFIGS:
        path = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
        assert os.path.exists(path), name
        d = json.load(open(path))
        # every source read once, every destination written once: traffic = algorithmic bytes within
        # a few ppm-to-permille (a summary far off means the wrong kernel's dispatches were counted)
        assert 0.999 <= d["traffic_over_algorithmic"] <= 1.01, (name, d["traffic_over_algorithmic"])
        assert d["algorithmic_bytes_per_launch"] == bench.algorithmic_bytes(bench.CONFIGS[name])
        assert all(os.path.exists(os.path.join(ROOT, s)) for s in d["source"]), d["source"]


def _csv(path, rows):
    cols = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for i, (k, c, v) in enumerate(rows):
            w.writerow({"Dispatch_Id": i, "Kernel_Name": k, "Counter_Name": c, "Counter_Value": v})


def test_traffic_tool_counts_only_the_configs_instantiation(tmp_path):
    """C2's process also launches C1's small ring steps (policy 0) and other configurations: only
    reduce_copy_kernel<7, 0, 2, 3, ...> may enter the C2 median."""
    c2 = "void nexr::reduce_copy_kernel<7, 0, 2, 3, 4, 256>(nexr::RCParams)"
    c1 = "void nexr::reduce_copy_kernel<7, 0, 2, 0, 4, 256>(nexr::RCParams)"
    c3 = "void nexr::reduce_copy_kernel<9, 0, 8, 3, 1, 1024>(nexr::RCParams)"
    fetch = [(c2, "FETCH_SIZE", 262144.0)] * 3 + [(c1, "FETCH_SIZE", 1000.0)] * 50 + [(c3, "FETCH_SIZE", 1179648.0)] * 5
    write = [(c2, "WRITE_SIZE", 262144.0)] * 3 + [(c1, "WRITE_SIZE", 2048.0)] * 50 + [(c3, "WRITE_SIZE", 262144.0)] * 5
    _csv(tmp_path / "f.csv", fetch)
    _csv(tmp_path / "w.csv", write)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), "--config", "c2", "--fetch",
                    str(tmp_path / "f.csv"), "--write", str(tmp_path / "w.csv"), "--out", str(out)], check=True,
                   capture_output=True, cwd=ROOT)
    d = json.load(open(out))
    assert d["dispatches"] == {"fetch_pass": 3, "write_pass": 3}
    assert d["traffic_over_algorithmic"] == 1.0


def test_ll_step_traffic_summary_reproduces_from_the_committed_counters():
    """profiles/r02s5_ll_pmc.txt is rebuilt from the committed counter collections by
    tools/ll_prof_summary.py, and every LL / LL128 / SIMPLE step moves its algorithmic bytes once."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ll_prof_summary
    p = lambda n: os.path.join(ROOT, "profiles", n)  # noqa: E731
    rows = ll_prof_summary.main(["--fetch", p("r02s5_ll_pmc_fetch.csv"), "--write", p("r02s5_ll_pmc_write.csv"),
                                 "--rate", p("r02s5_ll_pmc_rate.jsonl")])
    assert len(rows) == 15 and {r["proto"] for r in rows} == {"ll", "ll128", "simple"}
    assert all(0.999 <= r["traffic_over_alg"] <= 1.02 for r in rows), rows
    committed = open(p("r02s5_ll_pmc.txt")).read().split("\n")[1:]
    for r in rows:
        assert any(f"{r['read_bytes']:>13} {r['write_bytes']:>13}" in ln for ln in committed), r
