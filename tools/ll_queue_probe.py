"""C1 (fp32 sum all-reduce, 4 MiB per rank, 2 thread ranks on one GPU, device memory) with the LL and
LL128 protocols, host-sequenced (NEXR_LL_ASYNC=0), queued launches with a completion ticket every 4
steps (NEXR_LL_RUN=0) and device runs (the default; nexrRingCommGetQueued reports which), each in a
child process, and the SIMPLE ring beside them (round 6 also measured tickets every 1, 2 and 7 steps
with NEXR_LL_TICKET_EVERY, profiles/r06e_*, r06g_*); ms per call over 20 calls, every call exact. Run under
`rocprofv3 --kernel-trace` to see the steps' kernels (tuning harness).
    python tools/ll_queue_probe.py [--child]"""
import importlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import numpy as np
    import torch
    ring = importlib.import_module("nex-nccl_amd.ring")
    n, count = 2, 1 << 20
    rng = np.random.default_rng(1)
    x = [rng.integers(-1000, 1000, count).astype(np.float32) for _ in range(n)]
    expect = x[0] + x[1]
    send = [torch.from_numpy(v).cuda() for v in x]
    recv = [torch.zeros(count, dtype=torch.float32, device="cuda") for _ in range(n)]
    out = {}
    for name, proto in (("simple", ring.PROTO_SIMPLE), ("ll", ring.PROTO_LL), ("ll128", ring.PROTO_LL128)):
        with ring.RingComm(n, ring.DEVICE_MEMORY, 0, None, protocol=proto, timeout_ms=10000) as comm:
            comm.all_reduce([t.data_ptr() for t in send], [t.data_ptr() for t in recv], count, 7, 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                comm.all_reduce([t.data_ptr() for t in send], [t.data_ptr() for t in recv], count, 7, 0)
            ms = (time.perf_counter() - t0) / 20 * 1e3
            ok = all(np.array_equal(r.cpu().numpy(), expect) for r in recv)
            out[name] = {"ms_per_call": round(ms, 3), "exact": ok, "queued": comm.queued()}
    return out


if __name__ == "__main__":
    if "--child" in sys.argv:
        print(json.dumps(run()))
        sys.exit(0)
    res = {}
    for tag, env in (("host_sequenced", {"NEXR_LL_ASYNC": "0"}),
                     ("queued_ticket_every_4", {"NEXR_LL_RUN": "0"}), ("device_runs", {})):
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=300)
        res[tag] = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else p.stderr[-500:]
    print(json.dumps(res, indent=1))
