#!/usr/bin/env python3
"""nexrReduceCopyHost on pageable buffers (fp32 sum, K=2, M=1) from 256 KiB to 64 MiB per buffer,
per host path and small-call chunk size, each setting in a child process (knobs are read once).
1 warm + N timed calls, output checked against a + b. Tuning harness, not a test."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [256 << 10, 1 << 20, 4 << 20, 8 << 20, 16 << 20, 32 << 20, 64 << 20, 128 << 20, 256 << 20]
SETTINGS = {"pipeline only": {"NEXR_HOST_COPY_THREADS": "0"},
            "team (8 threads) from 32 MiB per call": {"NEXR_HOST_MT_MIN_BYTES": str(32 << 20)},
            "solo below 4 MiB per call, else pipeline": {"NEXR_HOST_MT_MIN_BYTES": str(1 << 60)},
            "team (16 threads) from 32 MiB per call": {"NEXR_HOST_MT_MIN_BYTES": str(32 << 20),
                                                      "NEXR_HOST_COPY_THREADS": "16"}}


def child():
    sys.path.insert(0, ROOT)
    import importlib
    import numpy as np
    nexr = importlib.import_module("nex-nccl_amd")
    nexr.lib()
    out = {}
    for b in SIZES:
        n = b // 4
        rng = np.random.default_rng(b)
        a, c = rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)
        o = np.empty_like(a)
        call = lambda: nexr.reduce_copy_ptrs([a.ctypes.data, c.ctypes.data], [o.ctypes.data], n, 7, 0, host=True)  # noqa
        call()
        reps = max(3, min(50, (64 << 20) // b))
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        dt = (time.perf_counter() - t0) / reps
        out[f"{b >> 10} KiB"] = {"us": round(dt * 1e6, 1), "GBps": round(3 * b / dt / 1e9, 2),
                                 "exact": bool(np.array_equal(o, a + c))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
        sys.exit(0)
    for name, env in SETTINGS.items():
        p = subprocess.run([sys.executable, __file__, "--child"], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **env))
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        print(json.dumps({"setting": name, **(json.loads(lines[-1]) if lines else {"error": p.stderr[-400:]})}),
              flush=True)
