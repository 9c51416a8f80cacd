#!/usr/bin/env python3
"""Summarise tools/run_dram_pmc.sh: per kernel (the stream-mix probe's k_streams<S,U,W> and the C3
bf16 reduce-copy), the median per-dispatch value of every counter and the derived figures:
average EA read/write request latency = *_LEVEL / requests (Little's law: LEVEL accumulates the
requests in flight every cycle), and DRAM credit stalls per request.
    python tools/dram_pmc_summary.py gpurun_out/dram_pmc > profiles/r02_dram_pmc_summary.txt"""
import csv
import os
import re
import statistics
import sys
from collections import defaultdict

csv.field_size_limit(sys.maxsize)


def load(path, rows):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        m = re.search(r"k_streams<(\d+), (\d+), (\d+)>", name)
        if m:
            key = f"streams S={m.group(1)} U={m.group(2)} W={m.group(3)}"
        elif "reduce_copy_kernel<9, 0, 8" in name:
            key = "C3 bf16 reduce_copy_kernel K=8"
        else:
            continue
        rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))


def main():
    d = sys.argv[1]
    rows = defaultdict(lambda: defaultdict(list))
    for f in sorted(os.listdir(d)):
        if f.endswith("_counter_collection.csv"):
            load(os.path.join(d, f), rows)
    print(f"{'kernel':<34} {'RDREQ':>10} {'WRREQ':>10} {'rd lat':>8} {'wr lat':>8} {'rd stall/req':>12} "
          f"{'wr stall/req':>12} {'wr EA stall/req':>15}")
    for k in sorted(rows):
        c = {n: statistics.median(v) for n, v in rows[k].items()}
        rd, wr = c.get("TCC_EA0_RDREQ", 0), c.get("TCC_EA0_WRREQ", 0)
        rl = c.get("TCC_EA0_RDREQ_LEVEL", 0) / rd if rd else 0
        wl = c.get("TCC_EA0_WRREQ_LEVEL", 0) / wr if wr else 0
        rs = c.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL", 0) / rd if rd else 0
        ws = c.get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL", 0) / wr if wr else 0
        we = c.get("TCC_EA0_WRREQ_STALL", 0) / wr if wr else 0
        print(f"{k:<34} {rd:>10.0f} {wr:>10.0f} {rl:>8.1f} {wl:>8.1f} {rs:>12.3f} {ws:>12.3f} {we:>15.3f}")
    print("\nlatencies in TCC cycles per request; stalls = cycles a DRAM-bound request waited for credits, per request")


if __name__ == "__main__":
    main()
