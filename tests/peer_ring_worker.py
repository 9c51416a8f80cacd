"""One rank of a process-per-rank peer ring (nexrPeerRingCommCreate / nexrPeerRing*).

Started by tests/test_peer_ring_gpu.py as a child process, one per rank. Every rank regenerates
all ranks' inputs from the seed, keeps its own, runs `calls` collectives of kind --coll on the same
communicator (for all-reduce the later ones in place, so step counters carry over between calls)
and saves the output of each call to <out>.<call>.npy.
"""
import argparse
import importlib
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    for name in ("rank", "n", "dt", "op", "count", "seed", "proto", "buff", "calls"):
        ap.add_argument(f"--{name}", type=int, required=True)
    ap.add_argument("--coll", default="allreduce",
                    choices=["allreduce", "allreduce_resident", "allreduce_mixed", "allreduce_guard", "reducescatter",
                             "allgather", "reduce", "broadcast", "sendrecv"])
    ap.add_argument("--root", type=int, default=0)
    ap.add_argument("--dt2", type=int, default=-1, help="allreduce_guard: the second call's datatype")
    ap.add_argument("--op2", type=int, default=-1, help="allreduce_guard: the second call's op (-1: --op)")
    ap.add_argument("--shm", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ring = importlib.import_module("nex-nccl_amd.ring")
    n_in = a.count * a.n if a.coll == "reducescatter" else a.count
    n_out = a.count * a.n if a.coll == "allgather" else a.count
    inputs = mg.gen_inputs(a.dt, a.n, n_in, a.seed, special=True)
    # Rank r drives GPU r mod (visible GPUs): on a node every neighbour pair of the ring sits on two
    # GPUs and each step's reduce-copy writes into the next rank's FIFO over xGMI; on a one-GPU box all
    # ranks share GPU 0 and the same IPC mappings stay on the device.
    ordinal = a.rank % torch.cuda.device_count()
    torch.cuda.set_device(ordinal)
    assert torch.cuda.current_device() == ordinal
    dev = torch.device("cuda", ordinal)
    send = torch.from_numpy(inputs[a.rank].copy()).to(dev)
    recv = torch.zeros(n_out, dtype=send.dtype, device=dev)
    torch.cuda.synchronize()
    resident = a.coll in ("allreduce_resident", "allreduce_mixed", "allreduce_guard")
    extras = resident or a.coll == "sendrecv"  # the opt-in extras library (include/nexr_extras.h)
    with ring.PeerRingComm(a.n, a.rank, a.shm, device=ordinal, buff_bytes=a.buff, protocol=a.proto,
                           timeout_ms=20000 if resident else 60000, extras=extras) as comm:
        with open(f"{a.out}.device", "w") as f:  # the GPU, the GPU count, and the step wait in effect
            f.write(f"{ordinal} {torch.cuda.device_count()} {comm.step_wait()}\n")
        if a.coll == "allreduce_guard":
            # Call 0 agrees the team on its (datatype, op) kernel; call 1 runs a kernel that keeps fewer
            # workgroups resident per CU. Record how call 1 ended (result code, 0 = success) and how long
            # it took: a rank must return, not wait for peers whose workgroups cannot be scheduled.
            comm.all_reduce_resident(send.data_ptr(), recv.data_ptr(), a.count, a.dt, a.op)
            np.save(f"{a.out}.0.npy", recv.cpu().numpy())
            # Every rank past call 0 before any starts call 1: a rank failing call 1 aborts the
            # communicator, and with it any rank still inside call 0.
            open(f"{a.out}.call0", "w").close()
            base = os.path.join(os.path.dirname(a.out), "rank")
            t_end = time.monotonic() + 60
            while not all(os.path.exists(f"{base}{q}.call0") for q in range(a.n)):
                assert time.monotonic() < t_end, "ranks did not all finish call 0"
                time.sleep(0.005)
            x = torch.from_numpy(mg.gen_inputs(a.dt2, a.n, a.count, a.seed + 1, special=True)[a.rank].copy()).to(dev)
            torch.cuda.synchronize()
            t0 = time.monotonic()
            try:
                comm.all_reduce_resident(x.data_ptr(), x.data_ptr(), a.count, a.dt2, a.op if a.op2 < 0 else a.op2)
                code = 0
            except Exception as e:  # NexrError carries the ncclResult_t value
                code = getattr(e, "code", -1)
            with open(f"{a.out}.guard", "w") as f:
                f.write(f"{code} {time.monotonic() - t0:.3f}\n")
            return 0
        if a.coll not in ("allreduce", "allreduce_resident", "allreduce_mixed"):
            for call in range(a.calls):
                if a.coll == "reducescatter":
                    comm.reduce_scatter(send.data_ptr(), recv.data_ptr(), a.count, a.dt, a.op)
                elif a.coll == "sendrecv":  # call c: a ring shift by c+1 (a self-copy when it wraps)
                    k = (call + 1) % a.n
                    comm.send_recv(send.data_ptr(), (a.rank + k) % a.n, recv.data_ptr(), (a.rank - k) % a.n,
                                   a.count * send.element_size())
                elif a.coll == "allgather":
                    comm.all_gather(send.data_ptr(), recv.data_ptr(), a.count, a.dt)
                elif a.coll == "reduce":
                    comm.reduce(send.data_ptr(), recv.data_ptr() if a.rank == a.root else 0, a.count, a.dt, a.op,
                                a.root)
                else:
                    comm.broadcast(send.data_ptr() if a.rank == a.root else 0, recv.data_ptr(), a.count, a.dt,
                                   a.root)
                np.save(f"{a.out}.{call}.npy", recv.cpu().numpy())
            return 0
        def all_reduce(call):  # allreduce_mixed alternates the host-sequenced and the resident form
            if a.coll == "allreduce_mixed":
                return comm.all_reduce_resident if call % 2 else comm.all_reduce
            return comm.all_reduce_resident if resident else comm.all_reduce
        all_reduce(0)(send.data_ptr(), recv.data_ptr(), a.count, a.dt, a.op)
        np.save(f"{a.out}.0.npy", recv.cpu().numpy())
        for call in range(1, a.calls):
            # in place on the previous result: out_c = allreduce(out_{c-1})
            all_reduce(call)(recv.data_ptr(), recv.data_ptr(), a.count, a.dt, a.op)
            np.save(f"{a.out}.{call}.npy", recv.cpu().numpy())
    return 0


if __name__ == "__main__":
    sys.exit(main())
