"""One rank of a process-per-rank peer ring (nexrPeerRingCommCreate / nexrPeerRingAllReduce).

Started by tests/test_peer_ring_gpu.py as a child process, one per rank. Every rank regenerates
all ranks' inputs from the seed, keeps its own, runs `calls` all-reduces on the same communicator
(the later ones in place, so step counters carry over between calls) and saves the output of each
call to <out>.<call>.npy.
"""
import argparse
import importlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    for name in ("rank", "n", "dt", "op", "count", "seed", "proto", "buff", "calls"):
        ap.add_argument(f"--{name}", type=int, required=True)
    ap.add_argument("--shm", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ring = importlib.import_module("nex-nccl_amd.ring")
    inputs = mg.gen_inputs(a.dt, a.n, a.count, a.seed, special=True)
    dev = torch.device("cuda:0")
    send = torch.from_numpy(inputs[a.rank].copy()).to(dev)
    recv = torch.zeros_like(send)
    torch.cuda.synchronize()
    with ring.PeerRingComm(a.n, a.rank, a.shm, device=0, buff_bytes=a.buff, protocol=a.proto,
                           timeout_ms=60000) as comm:
        comm.all_reduce(send.data_ptr(), recv.data_ptr(), a.count, a.dt, a.op)
        np.save(f"{a.out}.0.npy", recv.cpu().numpy())
        for call in range(1, a.calls):
            # in place on the previous result: out_c = allreduce(out_{c-1})
            comm.all_reduce(recv.data_ptr(), recv.data_ptr(), a.count, a.dt, a.op)
            np.save(f"{a.out}.{call}.npy", recv.cpu().numpy())
    return 0


if __name__ == "__main__":
    sys.exit(main())
