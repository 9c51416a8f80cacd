#!/usr/bin/env python3
"""Rates of the LL and LL128 protocol steps (nexrReduceCopyLL / nexrReduceCopyLL128)
next to the SIMPLE reduce-copy of the same shape, on one MI355X. Tuning harness, not a test.

Shapes are the primitives a ring step runs (reference src/device/prims_ll.h:285-335 and
prims_ll128.h:360-400): send (src -> peer), recvReduceSend (src + peer -> peer), recvReduceCopySend
(src + peer -> dst + peer), recvReduceCopy (src + peer -> dst), recvCopySend (peer -> dst + peer).
The recv wire is written once by a send step with flag F; every timed step reads it with flag F and
writes its own send wire with F + 1, so the recv polls never wait.

Algorithmic bytes per step, n = data bytes: user buffers n each; an LL wire 2n (a 16-B line per 8
data bytes, device.h:695-708); an LL128 wire ceil(n / 1920) * 2048 (16 lines of 128 B per 1920 data
bytes, device.h:730-738). Kernel time: HIP events on the launch stream, median of 7 blocks of R
launches after warm-up. fp32 sum."""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {  # name: (src, nRecv, dst, nSend)
    "send": (1, 0, 0, 1),
    "recvReduceSend": (1, 1, 0, 1),
    "recvReduceCopySend": (1, 1, 1, 1),
    "recvReduceCopy": (1, 1, 1, 0),
    "recvCopySend": (0, 1, 1, 1),
}
PEAK_GBS = 8000.0


def wire_bytes(proto: str, n: int) -> int:
    return 2 * n if proto == "ll" else -(-n // 1920) * 2048


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="32768,589824,4194304,67108864", help="data bytes per step")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--reps", type=int, default=0, help="launches per timed block (0 = by size)")
    args = ap.parse_args(argv)
    import torch
    nexr = importlib.import_module("nex-nccl_amd")
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    F = 7
    rows = []
    for n in [int(x) for x in args.sizes.split(",")]:
        ne = n // 4
        src = torch.rand(ne, device="cuda")
        dst = torch.empty(ne, device="cuda")
        reps = args.reps or max(5, min(200, (1 << 30) // max(n, 1) // 8))
        wires = {p: [torch.zeros(wire_bytes(p, n) // 8 + 16, dtype=torch.int64, device="cuda") for _ in range(2)]
                 for p in ("ll", "ll128")}
        # the recv wire of each protocol, written once with flag F
        nexr.reduce_copy_ll(src.data_ptr(), [], [], 0, [wires["ll"][0].data_ptr()], [F], ne, 7, 0, stream=sp)
        nexr.reduce_copy_ll128(src.data_ptr(), [], [], 0, [wires["ll128"][0].data_ptr()], [F], ne, 7, 0, stream=sp)
        torch.cuda.synchronize()
        peer = torch.empty(ne, device="cuda")
        out2 = torch.empty(ne, device="cuda")
        for name in args.shapes.split(","):
            hs, nr, hd, nsd = SHAPES[name]
            line = {"shape": name, "data_bytes": n, "reps": reps}
            for proto in ("ll", "ll128", "simple"):
                if proto == "simple":
                    ins = ([src.data_ptr()] if hs else []) + ([peer.data_ptr()] if nr else [])
                    outs = ([dst.data_ptr()] if hd else []) + ([out2.data_ptr()] if nsd else [])

                    def launch():
                        nexr.reduce_copy_ptrs(ins, outs, ne, 7, 0, 0, None, False, sp)
                    alg = (len(ins) + len(outs)) * n
                else:
                    fn = nexr.reduce_copy_ll if proto == "ll" else nexr.reduce_copy_ll128
                    rw, sw = wires[proto]
                    recv = [rw.data_ptr()] if nr else []
                    send = [sw.data_ptr()] if nsd else []

                    def launch(fn=fn, recv=recv, send=send):
                        fn(src.data_ptr() if hs else 0, recv, [F] * len(recv), dst.data_ptr() if hd else 0, send,
                           [F + 1] * len(send), ne, 7, 0, stream=sp)
                    alg = (hs + hd) * n + (nr + nsd) * wire_bytes(proto, n)
                for _ in range(3):
                    launch()
                meds = []
                for _ in range(7):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(reps):
                        launch()
                    e1.record(s)
                    e1.synchronize()
                    meds.append(e0.elapsed_time(e1) / reps * 1e3)
                meds.sort()
                us = meds[3]
                line[proto] = {"us": round(us, 2), "alg_bytes": alg, "GBps": round(alg / us / 1e3, 1),
                               "frac": round(alg / us / 1e3 / PEAK_GBS, 3)}
            rows.append(line)
            print(json.dumps(line), flush=True)
        del wires
    return rows


if __name__ == "__main__":
    main()
