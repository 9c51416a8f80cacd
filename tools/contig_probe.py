#!/usr/bin/env python3
"""Allocation kind vs reduce-copy rate (diagnostic for the per-set spread, DESIGN §6.3 (docs/HISTORY.md §6) round 3).

The placement probe (tools/placement_probe.py) found a per-allocation cost that no pointer shift
inside an allocation moves. If that cost is how fragmented the physical memory behind an
allocation is (page-table fragment size, hence translation reach), a physically contiguous
allocation should be at the fast end every time. This probe times the production kernel (through
the ABI, per-launch HIP events, cases interleaved round-robin) on buffer sets allocated three ways:
  torch   one torch allocation per buffer, as bench.py makes them;
  malloc  one hipMalloc per buffer;
  contig  one hipExtMallocWithFlags(hipDeviceMallocContiguous) per buffer.
`sets` sets of each kind, identical input bytes in every set; every output is compared with the
first set's at the end. Tuning harness, not a test; prints one JSON line per case and a summary."""
import argparse
import ctypes
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

nexr = importlib.import_module("nex-nccl_amd")
nexr.lib()
hip = nexr.hip_runtime()
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
HIP_CONTIGUOUS = 0x4  # hipDeviceMallocContiguous (hip_runtime_api.h)
D2D = 3  # hipMemcpyDeviceToDevice

CFG = {"c2": (torch.float32, 7, 2, 256 << 20), "c3_bf16": (torch.bfloat16, 9, 8, 256 << 20),
       "c3_f16": (torch.float16, 6, 8, 256 << 20), "c4_i32": (torch.int32, 2, 4, 64 << 20)}


def raw_alloc(nbytes, contiguous):
    p = ctypes.c_void_p()
    rc = (hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_CONTIGUOUS) if contiguous
          else hip.hipMalloc(ctypes.byref(p), nbytes))
    if rc != 0:
        raise RuntimeError(f"{'hipExtMallocWithFlags(contiguous)' if contiguous else 'hipMalloc'} = {rc}")
    return p.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CFG))
    ap.add_argument("--sets", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=12)
    a = ap.parse_args()
    dt, dtid, k, buf = CFG[a.config]
    esz = torch.empty((), dtype=dt).element_size()
    n = buf // esz
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ref = [(torch.rand(n, device="cuda", generator=g) * 2 - 1).to(dt) if dt.is_floating_point
           else torch.randint(-1000, 1000, (n,), dtype=dt, device="cuda", generator=g) for _ in range(k)]
    torch.cuda.synchronize()
    cases, keep, raw = [], [], []
    for kind in ("torch", "malloc", "contig"):
        for s in range(a.sets):
            if kind == "torch":
                bufs = [torch.empty(n, dtype=dt, device="cuda") for _ in range(k + 1)]
                for r, b in zip(ref, bufs):
                    b.copy_(r)
                keep.append(bufs)
                ptrs = [b.data_ptr() for b in bufs]
            else:
                ptrs = [raw_alloc(buf, kind == "contig") for _ in range(k + 1)]
                raw += ptrs
                for r, p in zip(ref, ptrs):
                    hip.hipMemcpy(p, r.data_ptr(), buf, D2D)
            cases.append({"label": f"{kind}{s}", "kind": kind, "sp": ptrs[:k], "dp": ptrs[k:]})
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    times = {c["label"]: [] for c in cases}
    for _ in range(2):
        for c in cases:
            nexr.reduce_copy_ptrs(c["sp"], c["dp"], n, dtid, 0, 0, None, False, h)
    for r in range(a.rounds):
        order = cases if r % 2 == 0 else list(reversed(cases))
        evs = []
        for c in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            nexr.reduce_copy_ptrs(c["sp"], c["dp"], n, dtid, 0, 0, None, False, h)
            e1.record(stream)
            evs.append((c["label"], e0, e1))
        torch.cuda.synchronize()
        for label, e0, e1 in evs:
            times[label].append(e0.elapsed_time(e1) * 1e3)
        print(f"[round {r + 1}/{a.rounds}]", file=sys.stderr, flush=True)
    # every output against the first set's (identical inputs everywhere)
    first = torch.empty(n, dtype=dt, device="cuda")
    hip.hipMemcpy(first.data_ptr(), cases[0]["dp"][0], buf, D2D)
    same = []
    for c in cases:
        o = torch.empty(n, dtype=dt, device="cuda")
        hip.hipMemcpy(o.data_ptr(), c["dp"][0], buf, D2D)
        same.append(bool(torch.equal(o, first)))
    alg = (k + 1) * buf
    summary = {}
    for c, ok in zip(cases, same):
        t = times[c["label"]]
        med = statistics.median(t)
        rec = {"probe": a.config, "case": c["label"], "kind": c["kind"], "median_us": round(med, 2),
               "min_us": round(min(t), 2), "max_us": round(max(t), 2), "frac": round(alg / med / 1e-6 / 8e12, 4),
               "same_output": ok}
        summary.setdefault(c["kind"], []).append(rec["median_us"])
        print(json.dumps(rec), flush=True)
    print(json.dumps({"probe": a.config, "summary_median_us_per_set": summary,
                      "kind_mean_frac": {kd: round(alg / (sum(v) / len(v)) / 1e-6 / 8e12, 4) for kd, v in summary.items()}}),
          flush=True)
    for p in raw:
        hip.hipFree(p)


if __name__ == "__main__":
    main()
