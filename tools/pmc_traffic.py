#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes into HBM bytes per launch of the reduce-copy kernel.

Usage (after the two separate passes):
    python tools/pmc_traffic.py --fetch gpurun_out/prof_fetch/r01_counter_collection.csv \
        --write gpurun_out/prof_write/r01_counter_collection.csv --config c2 --out profiles/pmc_c2.json

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM (gfx950): FETCH_SIZE (KiB) counts
exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores.
"""
import argparse
import csv
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def per_dispatch(path, counter, kernel_substr):
    vals = []
    for r in csv.DictReader(open(path)):
        if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def instantiation(cfg) -> str:
    """The exact kernel instantiation a configuration launches, reduce_copy_kernel<DT, OP, K, POL, ...>
    (the policy from the bytes the call streams, as pickPolicy in nexr_api.cpp), so that other launches
    in the same process (C1's small ring steps, the extra configurations) never enter the median."""
    streamed = (cfg["k"] + cfg["m"]) * cfg["buf_bytes"]
    pol = 3 if streamed >= (512 << 20) else (1 if streamed >= (64 << 20) else 0)
    dt = cfg["dt"]
    # round 6 routing (nexr_api.cpp routeKernel): signed Sum / Prod / PreMulSum / SumPostDiv run the
    # unsigned type's kernel (int8 -> uint8, int32 -> uint32, int64 -> uint64); Min / Max keep their own
    if cfg["op"] != 2 and dt in (0, 2, 4):
        dt += 1
    return f"nexr::reduce_copy_kernel<{dt}, {cfg['op']}, {cfg['k']}, {pol},"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--kernel", default=None, help="kernel-name substring (default: the config's instantiation)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[a.config]
    a.kernel = a.kernel or instantiation(cfg)
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not f or not w:
        raise SystemExit("no dispatches of the kernel found")
    fetch_b = statistics.median(f) * 1024 * 2  # gfx950: FETCH_SIZE = 1/2 of a wide streaming read
    write_b = statistics.median(w) * 1024
    alg = bench.algorithmic_bytes(cfg)
    out = {
        "config": a.config,
        "workload": cfg["workload"],
        "kernel": a.kernel,
        "dispatches": {"fetch_pass": len(f), "write_pass": len(w)},
        "fetch_size_kib_raw_median": statistics.median(f),
        "write_size_kib_raw_median": statistics.median(w),
        "read_bytes_per_launch": int(fetch_b),
        "write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((fetch_b + write_b) / alg, 5),
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), x1024 KiB->B; WRITE_SIZE x1024",
        "source": [os.path.relpath(a.fetch), os.path.relpath(a.write)],
    }
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
