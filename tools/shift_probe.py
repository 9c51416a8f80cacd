#!/usr/bin/env python3
"""Shifted-pointer probe (follow-up of tools/placement_probe.py, whose slab and hybrid sets showed that
the K = 8 rate depends on where the K + M buffers sit relative to one another, not on any one buffer).

The production kernel (nexrReduceCopy) is run over buffer sets allocated with slack, with the
destination pointer moved by D bytes, or source s moved by s * D bytes. Moving a pointer by D inside
its own allocation is what a schedule that writes (or reads stream s) D bytes "later" than the
others would present to the memory system: it predicts, before building one, what a skewed
schedule could gain. The outputs are not checked (shifted sources pair different elements):
timing harness only, never a parity claim. Per-launch HIP events, round-robin over cases."""
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

CFG = {"c2": (torch.float32, 7, 2, 256 << 20), "c3_bf16": (torch.bfloat16, 9, 8, 256 << 20),
       "c4_i32": (torch.int32, 2, 4, 64 << 20)}


def run_cases(cases, rounds, dtid, n):
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    times = {c[0]: [] for c in cases}
    for lab, sp, dp in cases:
        nexr.reduce_copy_ptrs(sp, dp, n, dtid, 0, 0, None, False, h)
    for r in range(rounds):
        evs = []
        for lab, sp, dp in (cases if r % 2 == 0 else cases[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            nexr.reduce_copy_ptrs(sp, dp, n, dtid, 0, 0, None, False, h)
            e1.record(stream)
            evs.append((lab, e0, e1))
        torch.cuda.synchronize()
        for lab, e0, e1 in evs:
            times[lab].append(e0.elapsed_time(e1) * 1e3)
    return {k: statistics.median(v) for k, v in times.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3_bf16,c2")
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--shifts", default="0,4096,16384,65536,262144,1048576,2097152,4194304,8388608,16777216")
    args = ap.parse_args()
    shifts = [int(x) for x in args.shifts.split(",")]
    slack = max(shifts) * 8 + 4096
    for name in args.configs.split(","):
        dt, dtid, k, buf = CFG[name]
        esz = torch.empty((), dtype=dt).element_size()
        n = buf // esz
        bpl = (k + 1) * buf
        sets = []
        for _ in range(args.sets):
            bufs = [torch.empty(buf + slack, dtype=torch.uint8, device="cuda") for _ in range(k + 1)]
            for b in bufs[:k]:
                b.view(torch.int8).random_(-8, 8)  # small integers: finite in every float type
            sets.append(bufs)
        torch.cuda.synchronize()
        for si, bufs in enumerate(sets):
            sp0 = [b.data_ptr() for b in bufs[:k]]
            dp0 = bufs[k].data_ptr()
            cases = []
            for d in shifts:
                cases.append((f"dst+{d}", sp0, [dp0 + d]))
                if d:
                    cases.append((f"src_s+s*{d}", [p + s * d for s, p in enumerate(sp0)], [dp0]))
            cases.append(("in_place_src0", sp0, [sp0[0]]))
            med = run_cases(cases, args.rounds, dtid, n)
            for lab, us in med.items():
                print(json.dumps({"probe": name, "set": si, "case": lab, "median_us": round(us, 2),
                                  "frac": round(bpl / us / 1e3 / 8000, 4)}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
