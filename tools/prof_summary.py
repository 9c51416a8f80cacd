#!/usr/bin/env python3
"""Summarise a `rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py` run against the
bench line it printed: per reduce-copy instantiation, the dispatch count and the mean / median
duration of its device-resident launches (launches over PCIe, the h2d_inclusive zero-copy calls, run
in milliseconds and are split off), and the headline kernel's timed-region mean beside the bench's own
HIP-event figure.

    python tools/prof_summary.py --trace <dir>/c2_kernel_trace.csv --bench <bench json line file> \
        --command "<the profiled command>" --out profiles/<tag>_summary.txt
"""
import argparse
import csv
import json
import statistics
import sys

csv.field_size_limit(sys.maxsize)

PCIE_NS = 2_000_000  # a device-resident launch of any bench configuration takes < 0.5 ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--command", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    line = json.loads([ln for ln in open(a.bench) if ln.startswith("{")][-1])
    groups = {}
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"]
        if "reduce_copy" not in name:
            continue
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        groups.setdefault(name, []).append((int(r["Start_Timestamp"]), d, r["VGPR_Count"], r["Grid_Size_X"]))
    out = [f"command: {a.command}"]
    head = None
    for name, ds in sorted(groups.items(), key=lambda kv: kv[1][0][0]):
        ds.sort()
        dev = [d for _, d, _, _ in ds if d < PCIE_NS]
        pcie = [d for _, d, _, _ in ds if d >= PCIE_NS]
        out.append(f"{name}: {len(ds)} dispatches ({len(dev)} device-resident, {len(pcie)} over PCIe); "
                   f"VGPRs {ds[0][2]}, grid {ds[0][3]} work-items")
        if dev:
            out.append(f"  device-resident: mean {statistics.mean(dev) / 1e3:.2f} us, "
                       f"median {statistics.median(dev) / 1e3:.2f} us, min {min(dev) / 1e3:.2f} us")
        if pcie:
            out.append(f"  over PCIe: mean {statistics.mean(pcie) / 1e6:.3f} ms")
        if head is None:
            head = (name, dev)
    if head and head[1]:
        steps, warm = line["steps"], line["warmup"]
        timed = head[1][warm:warm + steps]
        ev = line["roofline"]["avg_kernel_us"]
        mean = statistics.mean(timed) / 1e3
        out.append(f"headline kernel, the {len(timed)} timed launches: mean {mean:.2f} us "
                   f"(bench HIP events under the same command: {ev:.2f} us; ratio {mean / ev:.4f})")
    r = line["roofline"]
    out.append(f"bench line under rocprof: value {line['value']} GB/s, roofline.achieved {r['achieved']} GB/s, "
               f"frac {r['frac']}")
    for k, v in (line.get("extra_configs") or {}).items():
        out.append(f"  extra {k}: {v['avg_kernel_us']} us = {v['achieved']} GB/s ({v['frac']})")
    open(a.out, "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
