#!/usr/bin/env python3
"""bench.py — device-resident reduce-copy GB/s (BASELINE.json metric) on 1..8 MI355X.

One "step" = one nexrReduceCopy launch over one batch: the BASELINE configs[1] workload, fp32 sum,
K=2 inputs, M=1 output, 256 MiB per buffer, inputs already resident in HBM (synthetic uniform
[-1, 1) data). Buffers rotate over 3 sets (2.3 GiB) so no step re-reads the previous step's
Infinity-Cache-resident bytes. With N GPUs every rank runs its own independent 256 MiB chunk
(configs[4]: no data-path collective; the barrier and the max-over-ranks timer are harness only),
so value = N x bytes per step / max-over-ranks time (weak scaling).

    python bench.py                       # N=1, default steps
    torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W

Prints ONE JSON line on rank 0 (keys per the driver contract, plus `roofline`, `cpu_baseline`,
`h2d_inclusive`).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)

# datatype / op ids = ncclDataType_t / ncclDevRedOp_t
CONFIGS = {
    "c2": dict(workload="fp32 sum, 2-input reduce-copy, 256 MiB per buffer, device-resident", dt=7, dtype="f32",
               op=0, arg=0, k=2, m=1, buf_bytes=256 << 20),
    "c3_f16": dict(workload="fp16 sum, 8-input reduce-copy, 256 MiB per buffer, device-resident", dt=6,
                   dtype="f16", op=0, arg=0, k=8, m=1, buf_bytes=256 << 20),
    "c3_bf16": dict(workload="bf16 sum, 8-input reduce-copy, 256 MiB per buffer, device-resident", dt=9,
                    dtype="bf16", op=0, arg=0, k=8, m=1, buf_bytes=256 << 20),
    "c4_i32_min": dict(workload="int32 min, 4-input reduce-copy, 64 MiB per buffer", dt=2, dtype="int32", op=2,
                       arg=0x80000000, k=4, m=1, buf_bytes=64 << 20),
    "c4_i32_max": dict(workload="int32 max, 4-input reduce-copy, 64 MiB per buffer", dt=2, dtype="int32", op=2,
                       arg=0x7FFFFFFF, k=4, m=1, buf_bytes=64 << 20),
    "c4_i32_prod": dict(workload="int32 prod, 4-input reduce-copy, 64 MiB per buffer", dt=2, dtype="int32", op=1,
                        arg=0, k=4, m=1, buf_bytes=64 << 20),
    "c4_i8_min": dict(workload="int8 min, 4-input reduce-copy, 64 MiB per buffer", dt=0, dtype="int8", op=2,
                      arg=0x80, k=4, m=1, buf_bytes=64 << 20),
    "c4_i8_max": dict(workload="int8 max, 4-input reduce-copy, 64 MiB per buffer", dt=0, dtype="int8", op=2,
                      arg=0x7F, k=4, m=1, buf_bytes=64 << 20),
    "c4_i8_prod": dict(workload="int8 prod, 4-input reduce-copy, 64 MiB per buffer", dt=0, dtype="int8", op=1,
                       arg=0, k=4, m=1, buf_bytes=64 << 20),
}
ESZ = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2}
METRIC = "device-resident reduce-copy GB/s, fp32 sum, K-way fan-in, 1/2/4/8 MI355X"


def algorithmic_bytes(cfg) -> int:
    """Every src read once, every dst written once."""
    return (cfg["k"] + cfg["m"]) * cfg["buf_bytes"]


# ---- distributed plumbing (harness only: no data-path collective) -----------------------------
def local_device_index() -> int:
    """This rank's GPU: LOCAL_RANK, folded onto the visible devices (a launcher that gives every rank
    one visible GPU, or a rehearsal with more ranks than GPUs, still lands on a valid device)."""
    import torch
    return int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())


class Dist:
    def __init__(self, backend: str | None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = local_device_index() if backend == "nccl" else int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        self.backend = backend
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if backend == "nccl":
                import torch
                kw["device_id"] = torch.device("cuda", self.local_rank)
            dist.init_process_group(backend=backend, rank=self.rank, world_size=self.world, **kw)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, value: float, device=None) -> float:
        if not self.pg:
            return value
        import torch
        t = torch.tensor([value], dtype=torch.float64, device=device if self.backend == "nccl" else None)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def gather(self, values, device=None) -> list:
        """Every rank's `values` (a list of floats of one length), indexed by rank; harness only."""
        if not self.pg:
            return [list(values)]
        import torch
        dev = device if self.backend == "nccl" else None
        t = torch.tensor(values, dtype=torch.float64, device=dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.pg.all_gather(out, t)
        return [o.tolist() for o in out]

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def timed_steps(step, steps: int, warmup: int, sync, dist: Dist, device=None):
    """W untimed steps, then EXACTLY `steps` steps bracketed by barrier + sync on both sides.
    Returns (local seconds, max-over-ranks seconds)."""
    for i in range(warmup):
        step(i)
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    sync()
    t1 = time.perf_counter()
    dist.barrier()
    local = t1 - t0
    return local, dist.max(local, device)


# ---- CPU baseline: the oracle (C restatement) on a bounded sample ------------------------------
def cpu_baseline(cfg, seconds: float = 10.0, threads: int = 1):
    import numpy as np
    import oracle

    n = (32 << 20) // ESZ[cfg["dt"]]  # 32 MiB per buffer sample
    rng = np.random.default_rng(7)
    store = {0: np.uint8, 1: np.uint8, 2: np.uint32, 3: np.uint32, 4: np.uint64, 5: np.uint64, 6: np.uint16,
             7: np.float32, 8: np.float64, 9: np.uint16}[cfg["dt"]]
    if cfg["dt"] == 7:
        srcs = [(rng.random(n, dtype=np.float32) * 2 - 1) for _ in range(cfg["k"])]
    else:
        srcs = [rng.integers(0, 256, n * ESZ[cfg["dt"]], dtype=np.uint8).view(store) for _ in range(cfg["k"])]
    dsts = [np.empty_like(srcs[0]) for _ in range(cfg["m"])]
    oracle.reduce_copy(srcs, cfg["m"], cfg["dt"], cfg["op"], cfg["arg"], dsts=dsts, threads=threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.reduce_copy(srcs, cfg["m"], cfg["dt"], cfg["op"], cfg["arg"], dsts=dsts, threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gbs = reps * (cfg["k"] + cfg["m"]) * n * ESZ[cfg["dt"]] / el / 1e9
    return gbs, reps, el


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(config_name: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config_name}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-h2d", action="store_true")
    ap.add_argument("--no-xgmi", action="store_true", help="skip the xGMI peer-step probe (N > 1 only)")
    ap.add_argument("--events", choices=["launch", "region"], default="region",
                    help="HIP events around every launch (default) or only around the timed region")
    args = ap.parse_args(argv)

    import numpy as np
    import torch

    cfg = CONFIGS[args.config]
    local_rank = local_device_index()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # NEXR_BENCH_BACKEND=gloo: rehearse the N > 1 harness where RCCL cannot run (several ranks on one
    # GPU); the barrier and max-over-ranks timer are the only collectives either way.
    dist = Dist(os.environ.get("NEXR_BENCH_BACKEND", "nccl"))
    if dist.world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={dist.world}")
    pkg = importlib.import_module("nex-nccl_amd")
    pkg.lib()

    esz = ESZ[cfg["dt"]]
    n = cfg["buf_bytes"] // esz
    R = 3
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + dist.rank)
    sets = []
    for r in range(R):
        if cfg["dt"] in (6, 7, 9):
            tdt = {6: torch.float16, 7: torch.float32, 9: torch.bfloat16}[cfg["dt"]]
            srcs = [(torch.rand(n, device=dev, generator=g) * 2 - 1).to(tdt) for _ in range(cfg["k"])]
        else:
            srcs = [torch.randint(0, 256, (cfg["buf_bytes"],), dtype=torch.uint8, device=dev, generator=g)
                    for _ in range(cfg["k"])]
        dsts = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8, device=dev) for _ in range(cfg["m"])]
        sets.append(([s.data_ptr() for s in srcs], [d.data_ptr() for d in dsts], srcs, dsts))
    stream = torch.cuda.current_stream(dev)
    handle = stream.cuda_stream
    total = args.warmup + args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(total)]

    per_launch = args.events == "launch"

    def step(i):
        sp, dp, _, _ = sets[i % R]
        if per_launch or i == args.warmup:
            ev[i][0].record(stream)
        pkg.reduce_copy_ptrs(sp, dp, n, cfg["dt"], cfg["op"], cfg["arg"], None, False, handle)
        if per_launch or i == total - 1:
            ev[i][1].record(stream)

    local_s, max_s = timed_steps(step, args.steps, args.warmup, torch.cuda.synchronize, dist, dev)
    if per_launch:
        kernel_ms = [ev[args.warmup + i][0].elapsed_time(ev[args.warmup + i][1]) for i in range(args.steps)]
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    else:
        avg_kernel_s = ev[args.warmup][0].elapsed_time(ev[total - 1][1]) / args.steps / 1e3
    bytes_step = algorithmic_bytes(cfg)
    value = dist.world * bytes_step * args.steps / max_s / 1e9
    achieved = bytes_step / avg_kernel_s / 1e9
    traffic, traffic_src = load_traffic(args.config)
    # per-GPU rates beside the aggregate (every rank's own wall time and kernel time).
    ranks = dist.gather([local_s, avg_kernel_s], dev)

    result = None
    if dist.rank == 0:
        cpu = None
        h2d = None
        if dist.world == 1 and not args.no_cpu:
            gbs1, reps, el = cpu_baseline(cfg, args.cpu_seconds, threads=1)
            nthreads = min(16, os.cpu_count() or 1)
            gbsN, _, _ = cpu_baseline(cfg, max(2.0, args.cpu_seconds / 4), threads=nthreads)
            cpu = {"value": round(gbs1, 3), "unit": "GB/s", "cores": 1, "kind": "port",
                   "sample": f"oracle/nexr_oracle.c (C restatement of reduceCopy), same op/dtype/K/M, "
                             f"32 MiB per buffer x {reps} reps in {el:.1f} s on 1 thread of {cpu_model()}",
                   "all_cores": {"value": round(gbsN, 3), "cores": nthreads}}
        if dist.world == 1 and not args.no_h2d:
            h2d = h2d_inclusive(pkg, cfg, n)
        xgmi = xgmi_probe() if dist.world > 1 and not args.no_xgmi else None
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": dist.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_s / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": cfg["dtype"],
            "data": "synthetic (uniform [-1,1) generated on device; inputs resident in HBM)",
            "config": {"workload": cfg["workload"], "k_inputs": cfg["k"], "m_outputs": cfg["m"],
                       "bytes_per_buffer": cfg["buf_bytes"], "bytes_per_step_per_gpu": bytes_step,
                       "parallelism": f"independent chunks x{dist.world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "kernel": "nexr::reduce_copy_kernel", "avg_kernel_us": round(avg_kernel_s * 1e6, 2),
                         "timing": ("HIP events around every launch on its stream" if per_launch else
                                    "HIP events around the timed region on the launch stream / steps"),
                         "traffic_source": traffic_src},
            "cpu_baseline": cpu,
            "h2d_inclusive": h2d,
        }
        if dist.world > 1:
            result["per_gpu"] = per_gpu_summary(ranks, bytes_step, args.steps)
        if xgmi is not None:
            result["xgmi_probe"] = xgmi
        print(json.dumps(result), flush=True)
    dist.close()
    return result


def per_gpu_summary(ranks, bytes_step: int, steps: int) -> dict:
    """Per-rank wall and kernel rates of an N > 1 run: `ranks[r] = [wall seconds, kernel seconds per
    launch]`. `value` stays the aggregate (N x bytes / max wall); this shows how even the ranks were."""
    wall = [bytes_step * steps / w / 1e9 for w, _ in ranks]
    kern = [bytes_step / k / 1e9 if k > 0 else 0.0 for _, k in ranks]
    return {"value": round(sum(wall) / len(wall), 2), "unit": "GB/s",
            "wall_gbs": [round(x, 1) for x in wall], "kernel_gbs": [round(x, 1) for x in kern],
            "min_wall_gbs": round(min(wall), 2), "max_wall_gbs": round(max(wall), 2)}


def xgmi_probe(timeout_s: float = 150.0):
    """The peer-memory step over xGMI (tools/xgmi_probe.py), after the timed region, in a bounded
    subprocess: its outcome is reported, never allowed to fail the bench line."""
    import subprocess
    try:
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "xgmi_probe.py")], capture_output=True,
                           text=True, timeout=timeout_s)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode == 0 and lines:
            return json.loads(lines[-1])
        return {"error": f"exit {p.returncode}", "stderr": p.stderr[-300:]}
    except Exception as e:  # noqa: BLE001 - reported, not raised
        return {"error": repr(e)[:300]}


def h2d_inclusive(pkg, cfg, n, reps: int = 3):
    """Rate with the host<->device traffic included (nexrReduceCopyHost on host buffers).

    Pinned buffers take the zero-copy path (the kernel reads/writes host memory over PCIe, both
    directions at once); pageable buffers take the staged two-stream chunk pipeline."""
    import numpy as np
    import torch

    def run(srcs, dsts):
        sp = [s.data_ptr() if hasattr(s, "data_ptr") else s.ctypes.data for s in srcs]
        dp = [d.data_ptr() if hasattr(d, "data_ptr") else d.ctypes.data for d in dsts]
        pkg.reduce_copy_ptrs(sp, dp, n, cfg["dt"], cfg["op"], cfg["arg"], None, False, 0, host=True)
        t0 = time.perf_counter()
        for _ in range(reps):
            pkg.reduce_copy_ptrs(sp, dp, n, cfg["dt"], cfg["op"], cfg["arg"], None, False, 0, host=True)
        return (time.perf_counter() - t0) / reps

    pinned_s = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8).pin_memory() for _ in range(cfg["k"])]
    pinned_d = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8).pin_memory() for _ in range(cfg["m"])]
    for s in pinned_s:
        s.random_(0, 255)
    t_pin = run(pinned_s, pinned_d)
    del pinned_s, pinned_d
    rng = np.random.default_rng(3)
    page_s = [rng.integers(0, 256, cfg["buf_bytes"], dtype=np.uint8) for _ in range(cfg["k"])]
    page_d = [np.empty(cfg["buf_bytes"], dtype=np.uint8) for _ in range(cfg["m"])]
    t_page = run(page_s, page_d)
    alg = algorithmic_bytes(cfg)
    return {"value": round(alg / t_pin / 1e9, 2), "unit": "GB/s", "ms_per_call": round(t_pin * 1e3, 3),
            "path": "nexrReduceCopyHost, pinned host buffers: zero-copy kernel over PCIe Gen5 x16",
            "pageable": {"value": round(alg / t_page / 1e9, 2), "ms_per_call": round(t_page * 1e3, 3),
                         "path": "staged H2D -> kernel -> D2H, two-stream 8 MiB chunk pipeline"}}


if __name__ == "__main__":
    main()
