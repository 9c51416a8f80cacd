#!/usr/bin/env python3
"""Rates of the reduce-copy's pre-/post-op forms and call shapes beyond the bench's nine
configurations (PreMulSum / SumPostDiv and the single-rank path), 256 MiB per
buffer, device-resident, 3 rotating buffer sets, HIP events on the launch stream (median of 7 blocks
of 5 launches after 3 warm-up launches). Algorithmic bytes = (K + M) x 256 MiB. Tuning harness, not
a test (the same calls are checked bit-exactly by tests/test_reduce_copy_gpu.py and test_onerank).

    python tools/op_rates.py
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK_GBS = 8000.0
BUF = 256 << 20


def main():
    import torch
    nexr = importlib.import_module("nex-nccl_amd")
    DT, OP, RO = nexr.DataType, nexr.DevRedOp, nexr.RedOp
    s = torch.cuda.current_stream()
    tdt = {DT.Float32: torch.float32, DT.Float16: torch.float16, DT.Bfloat16: torch.bfloat16, DT.Int32: torch.int32}

    def bufs(dt, k, m):
        n = BUF // torch.empty((), dtype=tdt[dt]).element_size()
        mk = (lambda: torch.rand(n, device="cuda").to(tdt[dt])) if dt != DT.Int32 else \
            (lambda: torch.randint(-1000, 1000, (n,), dtype=torch.int32, device="cuda"))
        return n, [([mk() for _ in range(k)], [torch.empty(n, dtype=tdt[dt], device="cuda") for _ in range(m)])
                   for _ in range(3)]

    def timed(launch):
        for i in range(3):
            launch(i)
        meds = []
        for b in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(5):
                launch(b * 5 + i)
            e1.record(s)
            e1.synchronize()
            meds.append(e0.elapsed_time(e1) / 5 * 1e3)
        return sorted(meds)[3]

    cases = []
    # ncclAvg on one rank through nexrLaunchOneRank: PreMulSum by 1/nRanks on floats (K = 1, M = 1)
    for dt in (DT.Float32, DT.Bfloat16, DT.Float16):
        cases.append(("onerank avg (PreMulSum, K=1)", dt, 1, 1, "onerank", None))
    # ncclAvg over 8 ranks of integers: SumPostDiv, K = 2 (a ring step's recvReduceCopy) and K = 4
    cases.append(("SumPostDiv /8, K=2", DT.Int32, 2, 1, "postdiv", 8))
    cases.append(("SumPostDiv /8, K=4", DT.Int32, 4, 1, "postdiv", 8))
    # PreMulSum with the pre-op on both sources (a reduce step's user input + peer), K = 2
    cases.append(("PreMulSum x0.5 both srcs, K=2", DT.Float32, 2, 1, "premul", None))
    # a ring recvReduceCopySend shape: two destinations
    cases.append(("Sum K=2 M=2", DT.Float32, 2, 2, "sum", None))
    cases.append(("copy K=1 M=1", DT.Float32, 1, 1, "sum", None))
    rows = []
    for name, dt, k, m, kind, ranks in cases:
        n, sets = bufs(dt, k, m)
        if kind == "onerank":
            full = nexr.host_to_dev_red_op(RO.Avg, dt, 8)

            def launch(i, sets=sets, full=full, dt=dt, n=n):
                src, dst = sets[i % 3]
                nexr.launch_one_rank(dst[0].data_ptr(), src[0].data_ptr(), n, full, dt, s.cuda_stream)
        else:
            if kind == "postdiv":
                op, arg, pre, post = OP.SumPostDiv, (ranks << 1) | 1, None, True
            elif kind == "premul":
                bits = int(torch.tensor([0.5], dtype=torch.float32).view(torch.int32).item()) & 0xFFFFFFFF
                op, arg, pre, post = OP.PreMulSum, bits, [bits] * k, False
            else:
                op, arg, pre, post = OP.Sum, 0, None, False

            def launch(i, sets=sets, op=op, arg=arg, pre=pre, post=post, dt=dt, n=n):
                src, dst = sets[i % 3]
                nexr.reduce_copy_ptrs([t.data_ptr() for t in src], [t.data_ptr() for t in dst], n, dt, op, arg, pre,
                                      post, s.cuda_stream)
        us = timed(launch)
        alg = (k + m) * BUF
        row = {"case": name, "dtype": dt.name, "K": k, "M": m, "us": round(us, 2), "GBps": round(alg / us / 1e3, 1),
               "frac": round(alg / us / 1e3 / PEAK_GBS, 3)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del sets
        torch.cuda.empty_cache()
    return rows


if __name__ == "__main__":
    main()
