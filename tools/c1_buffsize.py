"""C1's host_registered leg by FIFO size (diagnostic, not product code).

The bench's C1 leg (bench.py c1_ring) runs the ring all-reduce of 4 MiB per rank over 2 emulated ranks
with the reference's default NCCL_BUFFSIZE (4 MiB: 512 KiB steps, 1 MiB slices, 6 steps per rank), in
host memory with the user buffers registered (nexrHostRegister) and the FIFOs from nexrHostMemAlloc.
This times the same call with larger FIFOs (buffBytes 8-32 MiB: fewer, larger zero-copy steps) to
measure how far the step size moves the PCIe-bound time, with the per-step split and an exact check.

    python tools/c1_buffsize.py > gpurun_out/c1_buffsize.jsonl
"""
import importlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    torch.cuda.init()
    nexr = importlib.import_module("nex-nccl_amd")
    ring = importlib.import_module("nex-nccl_amd.ring")
    n, count, reps = 2, 1 << 20, 30
    rng = np.random.default_rng(1)
    x = [rng.integers(-1000, 1000, count).astype(np.float32) for _ in range(n)]
    expect = x[0] + x[1]
    send, recv = [v.copy() for v in x], [np.zeros(count, np.float32) for _ in range(n)]
    handles = [nexr.host_register(a.ctypes.data, a.nbytes) for a in send + recv]
    try:
        for buff in (4 << 20, 8 << 20, 16 << 20, 32 << 20):
            with ring.RingComm(n, ring.HOST_MEMORY, buff, None, protocol=ring.PROTO_SIMPLE, timeout_ms=10000) as comm:
                sp, rp = [a.ctypes.data for a in send], [a.ctypes.data for a in recv]
                comm.all_reduce(sp, rp, count, 7, 0)
                nexr.host_path_stats(reset=True)
                t0 = time.perf_counter()
                for _ in range(reps):
                    comm.all_reduce(sp, rp, count, 7, 0)
                dt = (time.perf_counter() - t0) / reps
                hp = nexr.host_path_stats(reset=True)
            steps = max(1, hp["calls"])
            print(json.dumps({"buff_mib": buff >> 20, "ms_per_call": round(dt * 1e3, 3),
                              "steps_per_call": round(hp["calls"] / reps, 2),
                              "zero_copy": hp["zeroCopyCalls"] == hp["calls"],
                              **{f"{k}_us_per_step": round(hp[k + "Ns"] / steps / 1e3, 2) for k in ("launch", "wait")},
                              "exact": all(np.array_equal(r, expect) for r in recv)}), flush=True)
    finally:
        for h in handles:
            nexr.host_deregister(h)


if __name__ == "__main__":
    main()
