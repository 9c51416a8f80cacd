#!/usr/bin/env python3
"""xGMI probe for the peer-memory ring step: one process, GPUs 0 and 1, peer access
enabled both ways, and the reduce-copy kernel run on GPU 0 with one operand in GPU 1's HBM:

  local        srcs = [a0, b0] -> d0          (all on GPU 0: the HBM reference)
  remote read  srcs = [a0, b1] -> d0          (b1 streamed over xGMI into GPU 0's kernel)
  remote write srcs = [a0, b0] -> d1          (the NCCL_P2P_WRITE pattern: the result lands in the
                                                next GPU's memory, src/transport/p2p.cc:402)

fp32 sum, 256 MiB per buffer. Then the process-rank ring itself across the two GPUs
(`ring_processes`): two child processes, rank r on GPU r, each mapping the other's FIFO over IPC
(nexrPeerRingCommCreate), run the emulated ring all-reduce (C1's 4 MiB and 64 MiB of fp32 per rank,
SIMPLE; LL and LL128 at 4 MiB) with every step's reduce-copy writing into the peer GPU's HBM over
xGMI; every rank's result is checked exactly (integer-valued inputs). `--ring-all N` runs the same
ring with N processes on the first N GPUs; `--peer-step` runs only the three kernel legs (bench.py
runs each part as its own bounded subprocess). `--step-wait sync|word` sets NEXR_STEP_WAIT for the
ring's ranks: how each rank thread waits for its step before posting it (stream synchronisation, the
cross-GPU default, or the completion word); each rank reports the wait in effect, and bench.py runs
both so that a step-visibility fault (word wrong, sync right) is told apart from a link fault. Prints one JSON line; with fewer than two GPUs it prints a
"skipped" line and exits 0. bench.py runs it as bounded subprocesses when it drives more than one
GPU, so a failure here can never take the bench line down with it.
"""
from __future__ import annotations

import ctypes
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(peer_step_only: bool = False) -> int:
    import torch

    n_dev = torch.cuda.device_count()
    if n_dev < 2:
        print(json.dumps({"skipped": f"needs 2 GPUs, found {n_dev}"}), flush=True)
        return 0
    if not torch.cuda.can_device_access_peer(0, 1):
        print(json.dumps({"skipped": "GPU 0 cannot access GPU 1's memory"}), flush=True)
        return 0
    pkg = importlib.import_module("nex-nccl_amd")
    hip = pkg.hip_runtime()  # the runtime torch and libnexr share, not a second copy
    for a, b in ((0, 1), (1, 0)):
        torch.cuda.set_device(a)
        rc = hip.hipDeviceEnablePeerAccess(ctypes.c_int(b), ctypes.c_uint(0))
        if rc not in (0, 704):  # hipSuccess, hipErrorPeerAccessAlreadyEnabled
            print(json.dumps({"skipped": f"hipDeviceEnablePeerAccess({a}->{b}) = {rc}"}), flush=True)
            return 0
    hip.hipGetLastError()
    n = 64 << 20  # fp32 elements: 256 MiB per buffer
    torch.cuda.set_device(0)
    d0, d1 = torch.device("cuda", 0), torch.device("cuda", 1)
    g = torch.Generator(device=d0)
    g.manual_seed(5)
    a0 = torch.rand(n, device=d0, generator=g)
    b0 = torch.rand(n, device=d0, generator=g)
    b1 = b0.to(d1)
    o0 = torch.empty(n, device=d0)
    o1 = torch.empty(n, device=d1)
    torch.cuda.synchronize(d0)
    torch.cuda.synchronize(d1)
    stream = torch.cuda.current_stream(d0)

    def timed(srcs, dst, iters=10):
        for _ in range(2):
            pkg.reduce_copy_ptrs([s.data_ptr() for s in srcs], [dst.data_ptr()], n, 7, 0, 0, None, False,
                                 stream.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            pkg.reduce_copy_ptrs([s.data_ptr() for s in srcs], [dst.data_ptr()], n, 7, 0, 0, None, False,
                                 stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / iters / 1e3

    buf = n * 4
    out = {"gpus": [0, 1], "bytes_per_buffer": buf, "kernel": "nexr::reduce_copy_kernel fp32 sum K=2 M=1"}
    t = timed([a0, b0], o0)
    out["local"] = {"us": round(t * 1e6, 1), "alg_GBps": round(3 * buf / t / 1e9, 1)}
    t = timed([a0, b1], o0)
    ok_read = torch.equal(o0, a0 + b0)
    out["remote_read"] = {"us": round(t * 1e6, 1), "xgmi_GBps": round(buf / t / 1e9, 1),
                          "alg_GBps": round(3 * buf / t / 1e9, 1), "exact": bool(ok_read)}
    t = timed([a0, b0], o1)
    torch.cuda.synchronize(d1)
    ok_write = torch.equal(o1.to(d0), a0 + b0)
    out["remote_write"] = {"us": round(t * 1e6, 1), "xgmi_GBps": round(buf / t / 1e9, 1),
                           "alg_GBps": round(3 * buf / t / 1e9, 1), "exact": bool(ok_write)}
    if not peer_step_only:
        out["ring_processes"] = ring_processes()
        if os.environ.get("NEXR_XGMI_RESIDENT") != "1":
            print(json.dumps(out), flush=True)
            return 0
        try:
            out["resident_ring"] = resident_ring(min(n_dev, 8))
        except Exception as e:  # noqa: BLE001 - reported, never raised
            out["resident_ring"] = {"error": repr(e)[:300]}
    print(json.dumps(out), flush=True)
    return 0


def resident_ring(n_ranks: int, sizes=(1 << 22, 1 << 26, 1 << 28), channels=(1, 4)):
    """The ring all-reduce with every step inside one device-resident launch per GPU
    (nexrRingAllReduceResident): thread ranks of one process, rank r's buffers on GPU r, FIFO bytes and
    step counters crossing xGMI. fp32 sum of integer-valued inputs, every rank's result checked exactly;
    algbw = bytes per rank / time, busbw = algbw x 2(n-1)/n (the reference's convention)."""
    import time
    import torch
    ring = importlib.import_module("nex-nccl_amd.ring")
    nd = torch.cuda.device_count()  # rank r on GPU r (folded onto the visible GPUs when rehearsing)
    out = {"ranks": n_ranks, "gpus": [r % nd for r in range(n_ranks)]}
    for nch in channels:
        for nbytes in sizes:
            count = nbytes // 4
            xs = [torch.arange(count, dtype=torch.float32, device=f"cuda:{r % nd}").remainder_(1000) + r
                  for r in range(n_ranks)]
            ys = [torch.empty_like(x) for x in xs]
            for d in range(min(nd, n_ranks)):
                torch.cuda.synchronize(d)
            with ring.RingComm(n_ranks, ring.DEVICE_MEMORY, 0, n_channels=nch, timeout_ms=10000, extras=True) as comm:
                comm.all_reduce_resident([x.data_ptr() for x in xs], [y.data_ptr() for y in ys], count, 7, 0)
                iters = 10
                t0 = time.perf_counter()
                for _ in range(iters):
                    comm.all_reduce_resident([x.data_ptr() for x in xs], [y.data_ptr() for y in ys], count, 7, 0)
                dt = (time.perf_counter() - t0) / iters
            exact = all(torch.equal(y, (torch.arange(count, dtype=torch.float32, device=y.device).remainder_(1000)
                                        * n_ranks + n_ranks * (n_ranks - 1) // 2)) for y in ys)
            out[f"ch{nch}_{nbytes}"] = {"ms": round(dt * 1e3, 4), "algbw_GBps": round(nbytes / dt / 1e9, 2),
                                        "busbw_GBps": round(nbytes * 2 * (n_ranks - 1) / n_ranks / dt / 1e9, 2),
                                        "exact": bool(exact)}
            del xs, ys
    return out


PROTOCOLS = {"simple": 0, "ll": 1, "ll128": 2}
if os.environ.get("NEXR_XGMI_RESIDENT") == "1":  # beyond SURVEY §8: opt-in, needs the extras library
    PROTOCOLS["simple_resident"] = 0  # nexrPeerRingAllReduceResident
LL_COUNT = 1 << 20  # the LL protocols run C1's 4 MiB only (they move 2x / 16/15x the payload)


def ring_rank(rank: int, n_ranks: int, shm: str, counts) -> int:
    """One rank of the cross-GPU process ring (child process, GPU `rank`): the SIMPLE ring at every
    count, then the LL and LL128 rings at C1's size, one communicator per protocol. Every rank checks
    its own output exactly and prints its line."""
    import time
    import torch
    dev = rank % torch.cuda.device_count()  # GPU r; folded onto the visible GPUs when rehearsing
    torch.cuda.set_device(dev)
    ring = importlib.import_module("nex-nccl_amd.ring")
    out = {}
    waits = {}
    for pname, proto in PROTOCOLS.items():
        out[pname] = res = {}
        with ring.PeerRingComm(n_ranks, rank, f"{shm}_{pname}", device=dev, protocol=proto,
                               timeout_ms=30000, extras=pname == "simple_resident") as comm:
            waits[pname] = comm.step_wait()
            call = comm.all_reduce_resident if pname == "simple_resident" else comm.all_reduce
            for count in (counts if pname.startswith("simple") else [LL_COUNT]):
                x = torch.arange(count, dtype=torch.float32, device=f"cuda:{dev}").remainder_(1000) + rank
                y = torch.empty_like(x)
                exp = (torch.arange(count, dtype=torch.float32, device=f"cuda:{dev}").remainder_(1000) * n_ranks
                       + n_ranks * (n_ranks - 1) // 2)
                torch.cuda.synchronize()
                call(x.data_ptr(), y.data_ptr(), count, 7, 0)  # warm-up, connects the FIFOs
                iters = 5
                t0 = time.perf_counter()
                for _ in range(iters):
                    call(x.data_ptr(), y.data_ptr(), count, 7, 0)
                dt = (time.perf_counter() - t0) / iters
                res[str(count * 4)] = {"ms": round(dt * 1e3, 3), "algbw_GBps": round(count * 4 / dt / 1e9, 2),
                                       "exact": bool(torch.equal(y, exp))}
    print(json.dumps({"rank": rank, "gpu": dev, "step_wait": waits, "results": out}), flush=True)
    return 0


def ring_processes(n_ranks: int = 2, timeout_s: float = 60.0, counts: str = "1048576,16777216",
                   step_wait: str | None = None):
    """n_ranks child processes, rank r on GPU r mod visible, each mapping its successor's FIFO over IPC:
    the ring all-reduce at C1's 4 MiB (SIMPLE, LL, LL128) and 64 MiB (SIMPLE). Reports rank 0's timing
    and whether EVERY rank's output was exact. Children stay in this process's group, so a caller
    that kills the group on a timeout ends them too; on this function's own timeout they are killed."""
    import subprocess
    import uuid
    shm = f"/nexr_xgmi_{uuid.uuid4().hex[:12]}"
    env = dict(os.environ)
    if step_wait:
        env["NEXR_STEP_WAIT"] = step_wait
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--ring-rank", str(r), "--ranks",
                               str(n_ranks), "--shm", shm, "--counts", counts], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=env) for r in range(n_ranks)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout_s))
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        return {"error": "timeout", "ranks": n_ranks, "step_wait": step_wait or "default"}
    finally:
        for pname in PROTOCOLS:
            if os.path.exists(f"/dev/shm{shm}_{pname}"):
                os.unlink(f"/dev/shm{shm}_{pname}")
    if any(p.returncode != 0 for p in procs):
        return {"error": [p.returncode for p in procs], "stderr": [e[-300:] for _, e in outs],
                "step_wait": step_wait or "default"}
    lines = [json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]) for o, _ in outs]
    r0 = lines[0]["results"]
    exact_all = all(v["exact"] for ln in lines for proto in ln["results"].values() for v in proto.values())
    return {"per_protocol_bytes": r0, "exact_all_ranks": exact_all, "gpus": [ln["gpu"] for ln in lines],
            "step_wait": step_wait or "default",
            "step_wait_in_effect": sorted({w for ln in lines for w in ln.get("step_wait", {}).values()}),
            "ranks": f"{n_ranks} processes, rank r on GPU r, fp32 sum; SIMPLE at 4 and 64 MiB (and the "
                     "device-resident form with NEXR_XGMI_RESIDENT=1), LL and LL128 at 4 MiB; "
                     "timings of rank 0"}


if __name__ == "__main__":
    a = sys.argv
    if "--resident-only" in a:  # rehearsal of the resident ring alone: --resident-only N
        print(json.dumps(resident_ring(int(a[a.index("--resident-only") + 1]))), flush=True)
        sys.exit(0)
    wait = a[a.index("--step-wait") + 1] if "--step-wait" in a else None
    if "--ring-only" in a:  # the two-rank process ring alone (any number of GPUs)
        print(json.dumps(ring_processes(step_wait=wait,
                                        timeout_s=float(os.environ.get("NEXR_RING_ONLY_TIMEOUT", "35")))), flush=True)
        sys.exit(0)
    if "--ring-all" in a:  # the process ring over the first N GPUs (bench.py at N >= 3)
        n = int(a[a.index("--ring-all") + 1])
        print(json.dumps(ring_processes(n, timeout_s=float(os.environ.get("NEXR_RING_ALL_TIMEOUT", "50")),
                                        step_wait=wait)), flush=True)
        sys.exit(0)
    if "--ring-rank" in a:
        sys.exit(ring_rank(int(a[a.index("--ring-rank") + 1]), int(a[a.index("--ranks") + 1]),
                           a[a.index("--shm") + 1], [int(v) for v in a[a.index("--counts") + 1].split(",")]))
    sys.exit(main(peer_step_only="--peer-step" in a))
