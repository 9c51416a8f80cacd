"""Time the emulated collectives at the C1 size (fp32 sum, 4 MiB per rank, 2 and 4 ranks) on the
MI355X reduce-copy, per memory mode, protocol and collective, beside the same schedule run with the
CPU oracle as its reduce-copy (the reference's CPU path: every step on host cores). Tuning harness,
not a test; every result is checked against plain numpy arithmetic (integer-exact inputs)."""
import ctypes
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402

ring = importlib.import_module("nex-nccl_amd.ring")
count = 1 << 20  # 4 MiB of fp32 per rank
F32 = 7
L = oracle.lib()
cast = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
ORACLE_FNS = (cast(L.oracle_reduce_copy_fn), cast(L.oracle_reduce_copy_ll_fn), cast(L.oracle_reduce_copy_ll128_fn))


def run(n, mode_name, proto_name, coll, iters):
    proto = {"simple": ring.PROTO_SIMPLE, "ll": ring.PROTO_LL, "ll128": ring.PROTO_LL128}[proto_name]
    mode = ring.DEVICE_MEMORY if mode_name == "device" else ring.HOST_MEMORY
    pinned = mode_name == "host-pinned"
    rng = np.random.default_rng(n)
    # small integers: every sum order gives the same fp32 result, so numpy checks the schedule
    x = [rng.integers(-1000, 1000, count * n).astype(np.float32) for _ in range(n)]
    out_n = count * n if coll == "allgather" else count
    if coll == "sendrecv":  # ring shift of the first 4 MiB of every rank's input
        x = [v[:count].copy() for v in x]
    if mode == ring.DEVICE_MEMORY:
        send = [torch.from_numpy(v).cuda() for v in x]
        recv = [torch.zeros(out_n, dtype=torch.float32, device="cuda") for _ in range(n)]
        sp, rp = [t.data_ptr() for t in send], [t.data_ptr() for t in recv]
        torch.cuda.synchronize()
    elif pinned:  # page-locked user buffers: with the pinned FIFOs every step is one zero-copy kernel
        send = [torch.from_numpy(v).pin_memory() for v in x]
        recv = [torch.zeros(out_n, dtype=torch.float32).pin_memory() for _ in range(n)]
        sp, rp = [t.data_ptr() for t in send], [t.data_ptr() for t in recv]
    else:
        send, recv = x, [np.zeros(out_n, np.float32) for _ in range(n)]
        sp, rp = [v.ctypes.data for v in send], [v.ctypes.data for v in recv]
    fns = ORACLE_FNS if mode_name == "cpu-oracle" else (None, None, None)
    kw = dict(protocol=proto, ll_fn_address=fns[1], ll128_fn_address=fns[2], tree_ranks_per_node=1,
              n_channels=int(os.environ.get("RING_TIME_CHANNELS", "1")))
    with ring.RingComm(n, mode, 0, fns[0], extras=coll == "sendrecv", **kw) as comm:
        call = {"allreduce": lambda: comm.all_reduce(sp, rp, count, F32, 0),
                "tree": lambda: comm.tree_all_reduce(sp, rp, count, F32, 0),
                "reducescatter": lambda: comm.reduce_scatter(sp, rp, count, F32, 0),
                "allgather": lambda: comm.all_gather(sp, rp, count, F32),
                "sendrecv": lambda: comm.send_recv(sp, [(r + 1) % n for r in range(n)], rp,
                                                   [(r - 1) % n for r in range(n)], count * 4)}[coll]
        call()
        t0 = time.perf_counter()
        for _ in range(iters):
            call()
        dt = (time.perf_counter() - t0) / iters
    got = [r.cpu().numpy() if hasattr(r, "cpu") else r for r in recv]
    if coll in ("allreduce", "tree"):
        exp = [sum(v[:count] for v in x)] * n
    elif coll == "reducescatter":
        exp = [sum(v[k * count:(k + 1) * count] for v in x) for k in range(n)]
    elif coll == "sendrecv":
        exp = [x[(r - 1) % n] for r in range(n)]
    else:
        exp = [np.concatenate([v[:count] for v in x])] * n
    assert all(np.array_equal(g, e) for g, e in zip(got, exp)), (n, mode_name, proto_name, coll)
    return dt


print(f"{'ranks':>5} {'mode':<10} {'proto':<6} {'collective':<14} {'ms/call':>9} {'algbw GB/s':>11}")
for n in [int(v) for v in os.environ.get("RING_TIME_RANKS", "2,4").split(",")]:
    modes = os.environ.get("RING_TIME_MODES", "cpu-oracle,host,host-pinned,device").split(",")
    for mode_name, protos in (("cpu-oracle", ("simple",)), ("host", ("simple",)), ("host-pinned", ("simple",)),
                              ("device", ("simple", "ll", "ll128"))):
        if mode_name not in modes:
            continue
        for proto_name in protos:
            colls = ("allreduce", "tree", "reducescatter", "allgather")
            for coll in colls + (("sendrecv",) if proto_name == "simple" and ring.extras_available() else ()):
                iters = 3 if mode_name == "cpu-oracle" else 10
                dt = run(n, mode_name, proto_name, coll, iters)
                print(f"{n:>5} {mode_name:<10} {proto_name:<6} {coll:<14} {dt * 1e3:9.3f} {count * 4 / dt / 1e9:11.2f}",
                      flush=True)
