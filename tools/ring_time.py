"""Time the C1 configuration (fp32 sum all-reduce, 4 MiB per rank, 2 ranks) through the emulated
ring on the MI355X reduce-copy, per memory mode and protocol (tuning harness, not a test)."""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ring = importlib.import_module("nex-nccl_amd.ring")
count = 1 << 20
n = 2
rng = np.random.default_rng(0)
host_in = [rng.standard_normal(count).astype(np.float32) for _ in range(n)]
print(f"{'mode':<8} {'proto':<6} {'ms/allreduce':>13} {'algbw GB/s':>11}")
for mode_name, mode in (("host", ring.HOST_MEMORY), ("device", ring.DEVICE_MEMORY)):
    for proto_name, proto in (("simple", ring.PROTO_SIMPLE), ("ll", ring.PROTO_LL), ("ll128", ring.PROTO_LL128)):
        if mode == ring.HOST_MEMORY and proto != ring.PROTO_SIMPLE:
            continue  # LL/LL128 kernels poll device-visible lines: device memory only
        if mode == ring.HOST_MEMORY:
            send = host_in
            recv = [np.zeros_like(x) for x in host_in]
            sp = [x.ctypes.data for x in send]
            rp = [x.ctypes.data for x in recv]
        else:
            send = [torch.from_numpy(x).cuda() for x in host_in]
            recv = [torch.zeros_like(x) for x in send]
            sp = [x.data_ptr() for x in send]
            rp = [x.data_ptr() for x in recv]
        torch.cuda.synchronize()
        with ring.RingComm(n, mode, 0, protocol=proto) as comm:
            for _ in range(3):
                comm.all_reduce(sp, rp, count, 7, 0)
            iters = 20
            t0 = time.perf_counter()
            for _ in range(iters):
                comm.all_reduce(sp, rp, count, 7, 0)
            dt = (time.perf_counter() - t0) / iters
        out = recv[0] if mode == ring.HOST_MEMORY else recv[0].cpu().numpy()
        assert np.array_equal(out.view(np.uint32), (host_in[0] + host_in[1]).view(np.uint32))
        print(f"{mode_name:<8} {proto_name:<6} {dt * 1e3:13.3f} {count * 4 / dt / 1e9:11.2f}", flush=True)
