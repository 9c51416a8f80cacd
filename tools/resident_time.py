#!/usr/bin/env python3
"""Time the device-resident ring all-reduce (nexrRingAllReduceResident) against the host-sequenced
ring (nexrRingAllReduce) on the same communicator: fp32 sum, integer-valued inputs so every result
is checked exactly. One JSON line per (ranks, channels, bytes per rank). --colls adds the other
resident collectives (ReduceScatter / AllGather at the same bytes per rank of output / input,
Broadcast from rank 0), timed alone.

    python tools/resident_time.py [--sizes 4194304,67108864] [--ranks 2,4] [--channels 1,4]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4194304,67108864")
    ap.add_argument("--ranks", default="2,4")
    ap.add_argument("--channels", default="1,4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--colls", action="store_true")
    ap.add_argument("--tree", action="store_true", help="time the tree all-reduce (resident vs host) instead")
    args = ap.parse_args()
    import torch
    ring = importlib.import_module("nex-nccl_amd.ring")
    for n in [int(v) for v in args.ranks.split(",")]:
        for nch in [int(v) for v in args.channels.split(",")]:
            for nbytes in [int(v) for v in args.sizes.split(",")]:
                count = nbytes // 4
                xs = [torch.arange(count, dtype=torch.float32, device="cuda").remainder_(1000) + r for r in range(n)]
                ys = [torch.empty_like(x) for x in xs]
                exp = torch.arange(count, dtype=torch.float32, device="cuda").remainder_(1000) * n + n * (n - 1) // 2
                torch.cuda.synchronize()
                sp, rp = [x.data_ptr() for x in xs], [y.data_ptr() for y in ys]
                line = {"ranks": n, "channels": nch, "bytes_per_rank": nbytes}
                with ring.RingComm(n, ring.DEVICE_MEMORY, 0, n_channels=nch, timeout_ms=20000, extras=True) as comm:
                    pair = ((("resident", comm.tree_all_reduce_resident), ("host", comm.tree_all_reduce)) if args.tree
                            else (("resident", comm.all_reduce_resident), ("host", comm.all_reduce)))
                    line["algorithm"] = "tree" if args.tree else "ring"
                    for name, fn in pair:
                        for y in ys:
                            y.zero_()
                        torch.cuda.synchronize()
                        fn(sp, rp, count, 7, 0)
                        ok = all(torch.equal(y, exp) for y in ys)
                        iters = args.iters if name == "resident" else max(3, args.iters // 4)
                        t0 = time.perf_counter()
                        for _ in range(iters):
                            fn(sp, rp, count, 7, 0)
                        dt = (time.perf_counter() - t0) / iters
                        line[name] = {"ms": round(dt * 1e3, 4), "algbw_GBps": round(nbytes / dt / 1e9, 2),
                                      "busbw_GBps": round(nbytes * 2 * (n - 1) / n / dt / 1e9, 2), "exact": bool(ok)}
                line["speedup"] = round(line["host"]["ms"] / line["resident"]["ms"], 2)
                if args.colls:
                    line.update(other_colls(ring, n, nch, count, args.iters))
                print(json.dumps(line), flush=True)
                del xs, ys, exp
                torch.cuda.empty_cache()


def other_colls(ring, n, nch, count, iters):
    """ReduceScatter (recvcount = count), AllGather (sendcount = count) and Broadcast (count) resident."""
    import torch
    out = {}
    big = [torch.arange(count * n, dtype=torch.float32, device="cuda").remainder_(1000) + r for r in range(n)]
    small = [torch.empty(count, dtype=torch.float32, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()
    with ring.RingComm(n, ring.DEVICE_MEMORY, 0, n_channels=nch, timeout_ms=20000, extras=True) as comm:
        calls = {"reduce_scatter": lambda: comm.reduce_scatter_resident([b.data_ptr() for b in big],
                                                                        [s.data_ptr() for s in small], count, 7, 0),
                 "all_gather": lambda: comm.all_gather_resident([s.data_ptr() for s in small],
                                                                [b.data_ptr() for b in big], count, 7),
                 "broadcast": lambda: comm.broadcast_resident([small[0].data_ptr()] + [0] * (n - 1),
                                                              [s.data_ptr() for s in small], count, 7, 0)}
        for name, fn in calls.items():
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            dt = (time.perf_counter() - t0) / iters
            nbytes = count * 4 * (n if name != "broadcast" else 1)
            out[name] = {"ms": round(dt * 1e3, 4), "algbw_GBps": round(nbytes / dt / 1e9, 2)}
    return out


if __name__ == "__main__":
    main()
