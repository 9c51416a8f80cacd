#!/usr/bin/env python3
"""Sweep of nexrReduceCopyHost's copy-team path on pageable buffers (the C2 mix: 2 x 256 MiB in,
1 x 256 MiB out): threads x chunk bytes, each setting in a child process (the library reads the knobs
once), 1 warm + 3 timed calls, output checked against a + b. Tuning harness, not a test."""
import itertools
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import importlib
    import numpy as np
    nexr = importlib.import_module("nex-nccl_amd")
    nexr.lib()
    n = 64 << 20
    rng = np.random.default_rng(3)
    a = rng.random(n, dtype=np.float32)
    b = rng.random(n, dtype=np.float32)
    o = np.empty_like(a)
    call = lambda: nexr.reduce_copy_ptrs([a.ctypes.data, b.ctypes.data], [o.ctypes.data], n, 7, 0, host=True)  # noqa
    call()
    t0 = time.perf_counter()
    for _ in range(3):
        call()
    dt = (time.perf_counter() - t0) / 3
    ok = bool(np.array_equal(o, a + b))
    print(json.dumps({"ms": round(dt * 1e3, 3), "GBps": round(3 * n * 4 / dt / 1e9, 2), "exact": ok}), flush=True)


def main():
    rows = []
    for threads, chunk in itertools.product([1, 4, 8, 12, 16], [4 << 20, 16 << 20, 32 << 20]):
        if threads == 1 and chunk != 4 << 20:
            continue
        env = dict(os.environ, NEXR_HOST_COPY_THREADS=str(threads), NEXR_HOST_MT_CHUNK_BYTES=str(chunk))
        p = subprocess.run([sys.executable, __file__, "--child"], capture_output=True, text=True, timeout=120, env=env)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        r = json.loads(line[-1]) if line else {"error": p.stderr[-300:]}
        r.update(threads=threads, chunk_MiB=chunk >> 20, path="chunk pipeline" if threads == 1 else "copy team")
        print(json.dumps(r), flush=True)
        rows.append(r)


if __name__ == "__main__":
    child() if "--child" in sys.argv else main()
