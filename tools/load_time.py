"""First-launch cost of libnexr's code objects (diagnostic, not product code).

HIP loads a library's device code objects when its first kernel is launched. This times, in a
fresh process per sample, the first nexrReduceCopy call (fp32 sum K=2, 1 Mi elements, then a
synchronise) against the second, for each library given, samples interleaved across libraries.

    python tools/load_time.py nex-nccl_amd/libnexr.so xbin/libnexr_r04.so
"""
import ctypes
import json
import os
import subprocess
import sys
import time


def child(path: str) -> None:
    import torch
    torch.cuda.init()
    x = [torch.ones(1 << 20, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L = ctypes.CDLL(os.path.abspath(path))
    t1 = time.perf_counter()
    f = L.nexrReduceCopy
    vp = ctypes.c_void_p
    f.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_int,
                  ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, vp]
    srcs = (vp * 2)(x[0].data_ptr(), x[1].data_ptr())
    dsts = (vp * 1)(x[2].data_ptr())
    out = []
    for _ in range(2):
        t = time.perf_counter()
        assert f(2, srcs, 1, dsts, 1 << 20, 7, 0, 0, 0, None, 0, None) == 0
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t)
    assert float(x[2][0]) == 2.0
    print(json.dumps({"dlopen_ms": round((t1 - t0) * 1e3, 2), "first_call_ms": round(out[0] * 1e3, 2),
                      "second_call_ms": round(out[1] * 1e3, 3)}))


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    libs = sys.argv[1:]
    res = {p: [] for p in libs}
    for _ in range(5):
        for p in libs:
            r = subprocess.run([sys.executable, __file__, "--child", p], capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                print(r.stdout, r.stderr, file=sys.stderr)
                raise SystemExit(r.returncode)
            res[p].append(json.loads(r.stdout.strip().splitlines()[-1]))
    for p, rows in res.items():
        med = {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in rows[0]}
        print(json.dumps({"lib": p, "bytes": os.path.getsize(p), "median": med, "samples": rows}))


if __name__ == "__main__":
    main()
