#!/usr/bin/env python3
"""fp16 vs bf16 vs uint32 on the SAME buffers (diagnostic): the K = 8 configurations (C3) run their
fp16 and bf16 kernels on separately allocated sets in the bench line, so a difference between them
mixes placement with arithmetic. Here three rotating sets of 8 + 1 buffers of 256 MiB are filled once
with finite random bits (valid fp16 and bf16 alike), and nexrReduceCopy runs the same bytes as fp16 sum,
bf16 sum and uint32 sum (the cheapest fold), interleaved launch by launch; per-launch HIP events,
median per (type, set). Tuning harness, not a test."""
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

nexr = importlib.import_module("nex-nccl_amd")
nexr.lib()

BUF = 256 << 20
SETS, ROUNDS = 3, 12
TYPES = {"f16": (6, BUF // 2), "bf16": (9, BUF // 2), "u32": (3, BUF // 4)}


def main():
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    sets = []
    for _ in range(SETS):
        bufs = [torch.randint(0, 1 << 30, (BUF // 4,), dtype=torch.int32, device="cuda", generator=g)
                .bitwise_and_(0x3bff3bff) for _ in range(8)]  # |x| < 1: finite as fp16 and as bf16
        bufs.append(torch.empty(BUF // 4, dtype=torch.int32, device="cuda"))
        sets.append(bufs)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    cases = [(t, s) for s in range(SETS) for t in TYPES]
    times = {c: [] for c in cases}

    def launch(t, s):
        dt, n = TYPES[t]
        b = sets[s]
        nexr.reduce_copy_ptrs([x.data_ptr() for x in b[:8]], [b[8].data_ptr()], n, dt, 0, 0, None, False, h)

    for c in cases * 2:
        launch(*c)
    for r in range(ROUNDS):
        order = cases if r % 2 == 0 else cases[::-1]
        evs = []
        for c in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch(*c)
            e1.record(stream)
            evs.append((c, e0, e1))
        torch.cuda.synchronize()
        for c, e0, e1 in evs:
            times[c].append(e0.elapsed_time(e1) * 1e3)
    out = {}
    for (t, s), v in times.items():
        out.setdefault(t, []).append(round(statistics.median(v), 2))
    alg = 9 * BUF
    print(json.dumps({"median_us_per_set": out,
                      "frac_per_type": {t: round(alg / (sum(v) / len(v)) / 1e-6 / 8e12, 4) for t, v in out.items()},
                      "f16_over_u32": [round(a / b, 4) for a, b in zip(out["f16"], out["u32"])],
                      "bf16_over_u32": [round(a / b, 4) for a, b in zip(out["bf16"], out["u32"])]}), flush=True)


if __name__ == "__main__":
    main()
