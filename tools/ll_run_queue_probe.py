"""Do two runs of LL steps whose progress depends on each other (nexrReduceCopyLLSteps: B receives what
A sends, A waits for B's credits) complete when the process already holds many other streams, so that
HIP may put A's and B's streams on one hardware queue (GPU_MAX_HW_QUEUES, 4 by default)? For each
number of extra live streams, 20 trials of a 40-step exchange over 8 slots with a 300 ms timeout:
how many completed, how many timed out, and the slowest trial. Also the same with the two streams
made by hipExtStreamCreateWithCUMask (all CUs).
  python tools/ll_run_queue_probe.py > gpurun_out/ll_run_queue_probe.json"""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
nexr = importlib.import_module("nex-nccl_amd")


def exchange(sa, sb, slot=1 << 16, n=40, timeout_us=300_000):
    per = slot // 8
    a = torch.randn(n * per, device="cuda")
    b = torch.randn(n * per, device="cuda")
    out = torch.zeros_like(b)
    fifo = torch.zeros(slot * 8 + 4096, dtype=torch.uint8, device="cuda")
    f, h = fifo.data_ptr(), fifo.data_ptr() + slot * 8
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nexr.reduce_copy_ll_steps(b.data_ptr(), out.data_ptr(), [(f, h, 0)], [], slot,
                              [nexr.ll_step(0, k * per, 1, k * per, per, recv=True) for k in range(n)], 7, 0,
                              status=st.data_ptr(), timeout_us=timeout_us, stream=sb)
    nexr.reduce_copy_ll_steps(a.data_ptr(), 0, [], [(f, h, 0)], slot,
                              [nexr.ll_step(0, k * per, -1, 0, per, send=True) for k in range(n)], 7, 0,
                              status=st.data_ptr() + 4, timeout_us=timeout_us, stream=sa)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = int(st[0].item()) == 0 and int(st[1].item()) == 0 and torch.equal(out, a + b)
    return ok, dt


def main():
    hip = nexr.hip_runtime()
    res = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "trials": []}
    for extra in (0, 2, 4, 6, 8, 16):
        keep = [torch.cuda.Stream() for _ in range(extra)]
        for k in keep:  # make every extra stream's queue busy-able: one tiny kernel each
            with torch.cuda.stream(k):
                torch.zeros(1, device="cuda").add_(1)
        torch.cuda.synchronize()
        oks, worst = 0, 0.0
        for _ in range(20):
            sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
            ok, dt = exchange(sa.cuda_stream, sb.cuda_stream)
            oks += ok
            worst = max(worst, dt)
        res["trials"].append({"extra_streams": extra, "completed": oks, "of": 20, "worst_s": round(worst, 4)})
        print(json.dumps(res["trials"][-1]), file=sys.stderr, flush=True)
        del keep
    # streams with a CU mask (every CU)
    mk = hip.hipExtStreamCreateWithCUMask
    mk.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    mk.restype = ctypes.c_int
    mask = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
    keep = [torch.cuda.Stream() for _ in range(16)]
    oks, worst, err = 0, 0.0, 0
    for _ in range(20):
        s = [ctypes.c_void_p(), ctypes.c_void_p()]
        e = [mk(ctypes.byref(x), 8, mask) for x in s]
        if any(e):
            err = e
            break
        ok, dt = exchange(s[0].value, s[1].value)
        oks += ok
        worst = max(worst, dt)
        for x in s:
            hip.hipStreamDestroy(x)
    res["cu_mask_streams_with_16_extra"] = {"completed": oks, "of": 20, "worst_s": round(worst, 4), "err": err}
    # C1's LL all-reduce through the ring library (its rank streams have queues of their own) with the 16
    # extra streams still alive
    ring = importlib.import_module("nex-nccl_amd.ring")
    count = 1 << 20
    x = [torch.randint(-1000, 1000, (count,), device="cuda").float() for _ in range(2)]
    recv = [torch.zeros_like(v) for v in x]
    with ring.RingComm(2, ring.DEVICE_MEMORY, 0, None, 2000, ring.PROTO_LL) as comm:
        t0 = time.perf_counter()
        ok = True
        for _ in range(10):
            comm.all_reduce([v.data_ptr() for v in x], [v.data_ptr() for v in recv], count, 7, 0)
            ok = ok and all(torch.equal(r, x[0] + x[1]) for r in recv)
        res["ring_ll_with_16_extra"] = {"exact": bool(ok), "mode": comm.queued(),
                                        "ms_per_call": round((time.perf_counter() - t0) / 10 * 1e3, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
