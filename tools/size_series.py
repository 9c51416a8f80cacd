#!/usr/bin/env python3
"""C2-shaped reduce-copy (fp32 sum, K=2, M=1) at 64 MiB..2 GiB per buffer through the library with the
cache policy pinned (NEXR_POLICY=3, set before the library loads): kernel time vs bytes, to separate a
fixed per-launch cost (ramp-up, drain, kernel boundary) from the streaming rate. HIP events on the
launch stream, 3 rotating buffer sets, median of 7 blocks of 5 launches. Tuning harness, not a test."""
import importlib
import json
import os
import sys

os.environ.setdefault("NEXR_POLICY", "3")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    nexr = importlib.import_module("nex-nccl_amd")
    s = torch.cuda.current_stream()
    rows = []
    for mib in (64, 128, 256, 512, 1024, 2048):
        n = mib * (1 << 20) // 4
        sets = [[torch.rand(n, device="cuda") for _ in range(3)] for _ in range(3 if mib <= 1024 else 2)]
        def launch(i):
            a, b, o = sets[i % len(sets)]
            nexr.reduce_copy_ptrs([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n, 7, 0, 0, None, False, s.cuda_stream)
        for i in range(3):
            launch(i)
        meds = []
        for blk in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(5):
                launch(blk * 5 + i)
            e1.record(s)
            e1.synchronize()
            meds.append(e0.elapsed_time(e1) / 5 * 1e3)
        meds.sort()
        us = meds[len(meds) // 2]
        rows.append({"mib_per_buffer": mib, "us": round(us, 2), "GBps": round(3 * mib * (1 << 20) / us / 1e3, 1)})
        print(json.dumps(rows[-1]), flush=True)
        del sets
        torch.cuda.empty_cache()
    # the same 256 MiB call in blocks of 5, 40 and 200 back-to-back launches: does a longer stretch of
    # sustained HBM load run slower per launch (power / clock management), independent of size?
    n = 64 << 20
    sets = [[torch.rand(n, device="cuda") for _ in range(3)] for _ in range(3)]
    def launch256(i):
        a, b, o = sets[i % 3]
        nexr.reduce_copy_ptrs([a.data_ptr(), b.data_ptr()], [o.data_ptr()], n, 7, 0, 0, None, False, s.cuda_stream)
    for block in (5, 40, 200, 5, 40, 200):
        torch.cuda.synchronize()
        import time
        time.sleep(0.5)  # idle between stretches
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(block):
            launch256(i)
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / block * 1e3
        print(json.dumps({"mib_per_buffer": 256, "launches_back_to_back": block, "us_per_launch": round(us, 2),
                          "GBps": round(3 * 256 * (1 << 20) / us / 1e3, 1)}), flush=True)
    del sets
    # least-squares t = t0 + bytes / R over the rows
    xs = [3 * r["mib_per_buffer"] * (1 << 20) for r in rows]
    ys = [r["us"] for r in rows]
    mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    t0 = my - slope * mx
    print(json.dumps({"fit": "us = t0 + bytes / R", "t0_us": round(t0, 2), "R_GBps": round(1e-3 / slope, 1)}))


if __name__ == "__main__":
    main()
