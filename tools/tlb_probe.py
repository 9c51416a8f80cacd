#!/usr/bin/env python3
"""Which buffer sets run the K = 8 reduce-copy fast, and what differs in their address translation
(follow-up of tools/shift_probe.py: moving pointers inside their allocations changes nothing, the
allocation itself does). Phase 1 times `--sets` torch-allocated sets round-robin with HIP events and
prints each set's median; phase 2 launches set 0 `--reps` times, then set 1, ... so that a
rocprofv3 --pmc pass over this script can attribute its last sets x reps dispatches to the sets in
order. Timing harness, not a test."""
import argparse
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

nexr = importlib.import_module("nex-nccl_amd")
nexr.lib()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--dt", type=int, default=9)  # bf16
    ap.add_argument("--mib", type=int, default=256)
    a = ap.parse_args()
    esz = {9: 2, 6: 2, 7: 4, 2: 4}[a.dt]
    buf = a.mib << 20
    n = buf // esz
    sets = []
    for _ in range(a.sets):
        bufs = [torch.empty(buf, dtype=torch.uint8, device="cuda") for _ in range(a.k + 1)]
        for b in bufs[:a.k]:
            b.view(torch.int8).random_(-8, 8)
        sets.append(([b.data_ptr() for b in bufs[:a.k]], [bufs[a.k].data_ptr()], bufs))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    times = [[] for _ in sets]
    for r in range(a.rounds):
        evs = []
        for i, (sp, dp, _) in enumerate(sets):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            nexr.reduce_copy_ptrs(sp, dp, n, a.dt, 0, 0, None, False, h)
            e1.record(stream)
            evs.append((i, e0, e1))
        torch.cuda.synchronize()
        for i, e0, e1 in evs:
            times[i].append(e0.elapsed_time(e1) * 1e3)
    for i, t in enumerate(times):
        print(json.dumps({"set": i, "median_us": round(statistics.median(t), 2),
                          "addrs_hex": [hex(p) for p in sets[i][0] + sets[i][1]]}), flush=True)
    for i, (sp, dp, _) in enumerate(sets):  # phase 2: attributable dispatches
        for _ in range(a.reps):
            nexr.reduce_copy_ptrs(sp, dp, n, a.dt, 0, 0, None, False, h)
    torch.cuda.synchronize()
    print(json.dumps({"phase2": f"{a.sets} sets x {a.reps} launches, in set order"}), flush=True)


if __name__ == "__main__":
    main()
