#!/usr/bin/env python3
"""C1 (fp32 sum all-reduce, 4 MiB per rank, 2 emulated ranks, ring SIMPLE) in HOST memory — the
fork's own setting, where NEX "device memory" is host memory — under each nexrReduceCopyHost path,
each setting in a child process (the library reads its knobs once). Tuning harness, not a test."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTINGS = {"chunk pipeline (runtime H2D/D2H)": {"NEXR_HOST_COPY_THREADS": "0"},
            "default (solo zero-copy for <= 4 MiB calls)": {}}


def child():
    sys.path.insert(0, ROOT)
    import bench
    r = bench.c1_ring()
    print(json.dumps({k: r[k] for k in ("host_staged", "cpu_oracle", "device")}), flush=True)


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
        sys.exit(0)
    rounds = int(os.environ.get("C1_ROUNDS", "1"))
    for name, env in [kv for _ in range(rounds) for kv in SETTINGS.items()]:
        p = subprocess.run([sys.executable, __file__, "--child"], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **env))
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        print(json.dumps({"setting": name, **(json.loads(lines[-1]) if lines else {"error": p.stderr[-400:]})}),
              flush=True)
