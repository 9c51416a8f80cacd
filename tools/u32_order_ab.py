"""Launch order of the bench's uint32 comparator (`kernel_over_u32_sum`, DeviceWorkload.per_set).

Up to round 4 the comparator launched the uint32 sum right after the configuration's kernel on the same
buffer set. A C4 set is 4 x 64 MiB in + 64 MiB out = 320 MiB, and the MI355X's Infinity Cache holds
256 MB, so the uint32 sum may find part of the kernel's bytes still cached and run faster than it
would cold, which inflates the ratio. The "grouped" order launches the kernel on every set, then the
uint32 sum on every set, so no launch follows one on the same buffers. This tool runs both orders on
the same three sets of every C4 configuration (and C2 and C3 f16 as controls, whose sets are 768 MiB
and 2.25 GiB), alternating the orders, and prints the ratio under each. Not product code.

Result (profiles/r04f_u32_order_ab.txt, 4 x 12 rounds per order): the orders agree within the noise
on every configuration (mean ratios within 0.006, in both directions), so the paired order had no
cache bias; the bench now uses the grouped order anyway.

    python tools/u32_order_ab.py [repeats]
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    repeats = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    pkg = importlib.import_module("nex-nccl_amd")
    names = ["c4_i8_min", "c4_i8_max", "c4_i8_prod", "c4_i32_min", "c4_i32_max", "c4_i32_prod", "c2", "c3_f16"]
    out = {}
    for i, name in enumerate(names):
        cfg = bench.CONFIGS[name]
        wl = bench.DeviceWorkload(pkg, cfg, 0, seed=3000 + i)
        wl.run(6, 3, bench._Solo())  # warm the kernels and the sets
        r = {"paired": [], "grouped": []}
        for rep in range(repeats):
            for order in (("paired", "grouped") if rep % 2 == 0 else ("grouped", "paired")):
                r[order].append(wl.per_set(rounds=12, order=order)["kernel_over_u32_sum"])
        wl.free()
        mean = {k: round(sum(v) / len(v), 4) for k, v in r.items()}
        out[name] = {"paired": r["paired"], "grouped": r["grouped"], "mean_paired": mean["paired"],
                     "mean_grouped": mean["grouped"]}
        print(f"{name:12s} paired {mean['paired']:.4f} {r['paired']}  grouped {mean['grouped']:.4f} {r['grouped']}",
              flush=True)
    print(json.dumps({"repeats": repeats, "rounds_per_set": 12, "sets": 3, "configs": out}), flush=True)


if __name__ == "__main__":
    main()
