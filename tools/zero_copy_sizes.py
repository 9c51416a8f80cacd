"""Zero-copy reduce-copy over PCIe by call size (diagnostic, not product code).

C1's host_registered leg (bench.py c1_ring) runs 6 steps per rank of 1-2 MiB slices, each one
zero-copy kernel over PCIe on registered host memory. This times nexrReduceCopyHost on memory
registered with nexrHostRegister for the step shapes the ring issues (K=1 M=1 copy, K=2 M=1, K=2 M=2)
from 256 KiB to 64 MiB per buffer, one call at a time and two calls at once from two threads (the two
emulated ranks share one GPU and one PCIe link), with the host-path split per call.

    python tools/zero_copy_sizes.py > gpurun_out/zero_copy_sizes.txt
"""
import ctypes
import importlib
import json
import mmap
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="", help="comma-separated subset of the shape names")
    ap.add_argument("--mib", default="", help="comma-separated buffer sizes in KiB")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    nexr = importlib.import_module("nex-nccl_amd")
    maxb = 64 << 20
    regions = []
    for _ in range(2):  # one region per thread: 4 buffers of maxb bytes
        m = mmap.mmap(-1, 4 * maxb)
        a = np.frombuffer(m, dtype=np.uint8)
        a[:] = 1
        h = nexr.host_register(a.ctypes.data, a.nbytes)
        regions.append((m, a, h))
    shapes = {"copy K1 M1": (1, 1), "reduce K2 M1": (2, 1), "recvReduceCopySend K2 M2": (2, 2)}
    if args.shapes:
        shapes = {k: v for k, v in shapes.items() if k.split()[0] in args.shapes.split(",")}
    sizes = [int(x) << 10 for x in args.mib.split(",")] if args.mib else [256 << 10, 1 << 20, 2 << 20, 4 << 20,
                                                                         16 << 20, 64 << 20]
    out = []
    for name, (k, m_) in shapes.items():
        for b in sizes:
            n = b // 4

            def call(i):
                base = regions[i][1].ctypes.data
                nexr.reduce_copy_ptrs([base + j * b for j in range(k)], [base + (2 + j) * b for j in range(m_)], n, 7, 0,
                                      host=True)

            for threads in (1, 2):
                call(0)
                reps = max(4, min(200, (256 << 20) // (b * (k + m_))))
                nexr.host_path_stats(reset=True)
                t0 = time.perf_counter()
                if threads == 1:
                    for _ in range(reps):
                        call(0)
                else:
                    ts = [threading.Thread(target=lambda i=i: [call(i) for _ in range(reps)]) for i in range(2)]
                    for t in ts:
                        t.start()
                    for t in ts:
                        t.join()
                dt = (time.perf_counter() - t0) / reps
                st = nexr.host_path_stats(reset=True)
                calls = max(1, st["calls"])
                row = {"shape": name, "grid": os.environ.get("NEXR_GRID", "one-shot"), "bytes_per_buffer": b, "threads": threads, "us_per_call": round(dt * 1e6, 1),
                       "GBps": round(threads * (k + m_) * b / dt / 1e9, 1),
                       "zero_copy": st["zeroCopyCalls"] == st["calls"],
                       **{f"{x}_us": round(st[x + "Ns"] / calls / 1e3, 2) for x in ("classify", "launch", "wait")}}
                out.append(row)
                print(json.dumps(row), flush=True)
    for _, _, h in regions:
        nexr.host_deregister(h)


if __name__ == "__main__":
    main()
