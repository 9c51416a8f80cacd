#!/usr/bin/env python3
"""Time the device-resident ring all-reduce (nexrRingAllReduceResident) against the host-sequenced
ring (nexrRingAllReduce) on the same communicator: fp32 sum, integer-valued inputs so every result
is checked exactly. One JSON line per (ranks, channels, bytes per rank).

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
                with ring.RingComm(n, ring.DEVICE_MEMORY, 0, n_channels=nch, timeout_ms=20000) as comm:
                    for name, fn in (("resident", comm.all_reduce_resident), ("host", comm.all_reduce)):
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
                print(json.dumps(line), flush=True)
                del xs, ys, exp
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
