#!/usr/bin/env python3
"""bench.py — device-resident reduce-copy GB/s (BASELINE.json metric) on 1..8 MI355X.

One "step" = one nexrReduceCopy launch over one batch: the BASELINE configs[1] workload, fp32 sum,
K=2 inputs, M=1 output, 256 MiB per buffer, inputs already resident in HBM (synthetic uniform
[-1, 1) data). Buffers rotate over 3 sets (2.3 GiB) so no step re-reads the previous step's
Infinity-Cache-resident bytes. With N GPUs every GPU runs its own independent 256 MiB chunk
(configs[4], C5: no data-path collective and no RCCL), so value = N x bytes per step / max time
(weak scaling). Two ways to drive N GPUs, both measuring the same thing:

    python bench.py                                    # N=1 (+ C3/C4 extra configs, CPU baseline)
    torchrun --nproc-per-node N bench.py --gpus N      # one process per GPU; gloo (CPU) barrier/max
    python bench.py --gpus N                           # one process: nexrReduceCopyMultiDeviceSets,
                                                       #   a host thread + stream per GPU
Either N > 1 way also times an N=1 leg on GPU 0 in the same run, and every GPU alone, and reports
them beside the aggregate under `c5`.

Prints ONE JSON line on rank 0 (keys per the driver contract, plus `roofline`, `cpu_baseline`,
`h2d_inclusive`, `extra_configs` / `c1_ring` at N=1 and `per_gpu` / `c5` / `xgmi_probe` /
`phase_s` at N>1).
"""
from __future__ import annotations

import argparse
import contextlib
import importlib
import json
import os
import sys
import time

_T0 = time.perf_counter()  # process start (before torch): every N > 1 line reports its phases from here
ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
REF_CPU_GBS_SURVEY = 1.79  # the compiled reference reduceCopy, fp32 sum K=2, 1 core

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
EXTRA_ORDER = ["c3_f16", "c3_bf16", "c4_i32_min", "c4_i32_max", "c4_i32_prod", "c4_i8_min", "c4_i8_max",
               "c4_i8_prod"]
ESZ = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2}
FANOUT_SETS = 3  # rotating buffer sets per GPU, in every leg (N = 1 line, torchrun ranks, fan-out)
METRIC = "device-resident reduce-copy GB/s, fp32 sum, K-way fan-in, 1/2/4/8 MI355X"
KERNEL = "nexr::reduce_copy_kernel"
DATA = "synthetic (uniform [-1,1) generated on device; inputs resident in HBM)"


def algorithmic_bytes(cfg) -> int:
    """Every src read once, every dst written once."""
    return (cfg["k"] + cfg["m"]) * cfg["buf_bytes"]


# ---- harness plumbing (no data-path collective) ------------------------------------------------
def local_device_index() -> int:
    """This rank's GPU: LOCAL_RANK, folded onto the visible devices (a launcher that gives every rank
    one visible GPU, or a rehearsal with more ranks than GPUs, still lands on a valid device)."""
    import torch
    return int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())


@contextlib.contextmanager
def stdout_to_stderr():
    """Route fd 1 to fd 2 for the duration (native libraries print there too), so that rank 0's
    stdout carries exactly the one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class Dist:
    """Barrier, max and gather over the ranks of a torchrun launch. The default backend is gloo: the
    harness needs only host-side synchronisation (each rank synchronises its own GPU first), so the
    multi-GPU line never depends on RCCL (north_star: no RCCL on this path). NEXR_BENCH_BACKEND=nccl
    selects RCCL for the harness collectives instead."""

    def __init__(self, backend: str | None = "gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.pg = None
        self.backend = backend
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if backend == "nccl":
                import torch
                kw["device_id"] = torch.device("cuda", local_device_index())
            import datetime
            # 10 minutes: longer than any leg a rank may wait through (rank 0's xGMI probes are bounded
            # at ~4 minutes), far shorter than the 30-minute default should a rank ever hang
            kw["timeout"] = datetime.timedelta(minutes=10)
            with stdout_to_stderr():  # gloo prints its "[Gloo] Rank r is connected to ..." lines on fd 1
                dist.init_process_group(backend=backend, rank=self.rank, world_size=self.world, **kw)
                dist.barrier()
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def _dev(self, device):
        return device if self.backend == "nccl" else None

    def max(self, value: float, device=None) -> float:
        if not self.pg:
            return value
        import torch
        t = torch.tensor([value], dtype=torch.float64, device=self._dev(device))
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def gather(self, values, device=None) -> list:
        """Every rank's `values` (a list of floats of one length), indexed by rank; harness only."""
        if not self.pg:
            return [list(values)]
        import torch
        t = torch.tensor(values, dtype=torch.float64, device=self._dev(device))
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.pg.all_gather(out, t)
        return [o.tolist() for o in out]

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


class _Solo:
    """A one-rank stand-in for Dist (the N=1 legs and the extra configs)."""
    world, rank = 1, 0

    def barrier(self):
        pass

    def max(self, value, device=None):
        return value


def timed_steps(step, steps: int, warmup: int, sync, dist, device=None):
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


# ---- one configuration on one GPU --------------------------------------------------------------
def comparator_sequence(ns: int, rounds: int, order: str) -> list:
    """The per-set comparator's launches as (0 = the configuration's kernel | 1 = the uint32 sum, set):
    "grouped" runs the kernel on every set, then the uint32 sum on every set, so with two or more sets
    no launch follows one on the same buffers; "paired" runs both back to back on each set."""
    if order == "paired":
        return [(kd, i % ns) for i in range(rounds * ns) for kd in (0, 1)]
    if order == "grouped":
        return [(kd, j) for _ in range(rounds) for kd in (0, 1) for j in range(ns)]
    raise ValueError(f"order {order!r}")


class DeviceWorkload:
    """R rotating buffer sets of one configuration on one GPU, and the timed launch loop over them."""

    def __init__(self, pkg, cfg, device_index: int, seed: int, sets: int = 3):
        import torch
        self.pkg, self.cfg = pkg, cfg
        self.dev = torch.device("cuda", device_index)
        self.n = cfg["buf_bytes"] // ESZ[cfg["dt"]]
        g = torch.Generator(device=self.dev)
        g.manual_seed(seed)
        self.sets = []
        with torch.cuda.device(self.dev):
            for _ in range(sets):
                if cfg["dt"] in (6, 7, 9):
                    tdt = {6: torch.float16, 7: torch.float32, 9: torch.bfloat16}[cfg["dt"]]
                    srcs = [(torch.rand(self.n, device=self.dev, generator=g) * 2 - 1).to(tdt)
                            for _ in range(cfg["k"])]
                else:
                    srcs = [torch.randint(0, 256, (cfg["buf_bytes"],), dtype=torch.uint8, device=self.dev,
                                          generator=g) for _ in range(cfg["k"])]
                dsts = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8, device=self.dev) for _ in range(cfg["m"])]
                self.sets.append(([s.data_ptr() for s in srcs], [d.data_ptr() for d in dsts], srcs, dsts))
            self.stream = torch.cuda.current_stream(self.dev)
        self.handle = self.stream.cuda_stream

    def work(self, i: int = 0):
        sp, dp, _, _ = self.sets[i % len(self.sets)]
        return self.pkg.make_work(sp, dp, self.n, self.cfg["arg"])

    def per_set(self, rounds: int = 12, order: str = "grouped") -> dict:
        """After the timed region (and after check_exact: it overwrites the outputs): `rounds` launches
        per set, with HIP events around every launch on the launch stream; the average kernel time of
        each set and where its buffers sit (the same kernel ran one set of C3 at 0.81-0.83
        of peak and the other two at 0.75-0.77). Beside them, the same bytes as a uint32 sum (the
        cheapest fold, v_add_u32, at the uint32 kernel's own geometry: the configuration's, except that
        the 16-bit K = 8 kernels run 1 x 1024 lanes and the uint32 one 4 x 256) on the same buffers: the
        rate this placement gives the same K + M streams, so `kernel_over_u32_sum` says what the
        configuration's arithmetic costs over the bare streams. `order` (comparator_sequence):
        "grouped", the default since round 4, never launches on the buffers the previous launch used;
        "paired" ran the uint32 sum right after the kernel on the same set. The two give the same ratios
        within +-0.6 % on every configuration (profiles/r04f_u32_order_ab.txt): the nt loads leave no
        usable bytes of a set in the Infinity Cache."""
        import torch
        cfg, ns = self.cfg, len(self.sets)
        n32 = cfg["buf_bytes"] // 4
        evs = []
        with torch.cuda.device(self.dev):
            # untimed launches first: the first launch after the GPU idled runs a few % slow and would
            # otherwise always land on set 0, and the uint32 kernel's first launch loads its code object
            sp, dp, _, _ = self.sets[-1]
            self.pkg.reduce_copy_ptrs(sp, dp, self.n, cfg["dt"], cfg["op"], cfg["arg"], None, False, self.handle)
            self.pkg.reduce_copy_ptrs(sp, dp, n32, 3, 0, 0, None, False, self.handle)
            kinds = (("kernel", self.n, cfg["dt"], cfg["op"], cfg["arg"]), ("u32", n32, 3, 0, 0))
            for kd, j in comparator_sequence(ns, rounds, order):
                kind, n, dt, op, arg = kinds[kd]
                sp, dp, _, _ = self.sets[j]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(self.stream)
                self.pkg.reduce_copy_ptrs(sp, dp, n, dt, op, arg, None, False, self.handle)
                e1.record(self.stream)
                evs.append((kind, j, e0, e1))
            torch.cuda.synchronize(self.dev)
        us = {"kernel": [[] for _ in range(ns)], "u32": [[] for _ in range(ns)]}
        for kind, k, e0, e1 in evs:
            us[kind][k].append(e0.elapsed_time(e1) * 1e3)
        mean = lambda v: sum(v) / len(v)  # noqa: E731
        ker, u32 = [mean(u) for u in us["kernel"]], [mean(u) for u in us["u32"]]
        lo = min(p for sp, dp, _, _ in self.sets for p in sp + dp)
        return {"per_set_us": [round(x, 2) for x in ker],
                "per_set_frac": [round(algorithmic_bytes(cfg) / x / 1e3 / PEAK_HBM_GBS, 4) for x in ker],
                "per_set_launches": rounds, "per_set_order": order,
                "per_set_buffers_mib": [[round((p - lo) / (1 << 20), 3) for p in sp + dp] for sp, dp, _, _ in self.sets],
                "same_bytes_u32_sum_per_set_us": [round(x, 2) for x in u32],
                "kernel_over_u32_sum": round(mean(ker) / mean(u32), 4)}

    def check_exact(self, i: int, blocks: int = 256, block: int = 4096) -> dict:
        """Test infrastructure, outside every timed region: the output of set `i` (every set holds the
        output of its last launch; the inputs never change) against the CPU oracle, bit for bit, on a
        strided sample of whole runs of elements (`blocks` runs of `block` spread over the buffer, plus
        the first and the last run: >= 1 Mi elements), or on all of it when it is smaller."""
        import numpy as np
        import torch
        import oracle
        cfg, n, esz = self.cfg, self.n, ESZ[self.cfg["dt"]]
        _, _, srcs, dsts = self.sets[i % len(self.sets)]
        if n <= block * (blocks + 2):
            starts = [0]
            block = n
        else:
            starts = sorted({0, n - block} | {int(x) for x in np.linspace(0, n - block, blocks)})

        def sample(t):
            b = t.view(torch.uint8)
            return torch.cat([b[s * esz:(s + block) * esz] for s in starts]).cpu().numpy()

        on_gpu = self.dev.type == "cuda"
        with torch.cuda.device(self.dev) if on_gpu else contextlib.nullcontext():
            if on_gpu:
                torch.cuda.synchronize(self.dev)
            got = [sample(d) for d in dsts]
            ins = [sample(s) for s in srcs]
        exp = oracle.reduce_copy(ins, cfg["m"], cfg["dt"], cfg["op"], cfg["arg"])
        ok = all(np.array_equal(g, e.view(np.uint8)) for g, e in zip(got, exp))
        return {"exact": bool(ok), "checked_elements": len(starts) * block, "checked_set": i % len(self.sets),
                "check": "bit-exact vs the C oracle (oracle/nexr_oracle.c) on a strided sample of the last "
                         "launch's output, after the timed region"}

    def run(self, steps: int, warmup: int, dist, per_launch: bool = False):
        """Returns (local wall s, max-over-ranks wall s, average kernel s from HIP events recorded on
        the launch stream around the timed region, or around every launch)."""
        import torch
        cfg, total = self.cfg, warmup + steps
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(total)]

        def step(i):
            sp, dp, _, _ = self.sets[i % len(self.sets)]
            if per_launch or i == warmup:
                ev[i][0].record(self.stream)
            self.pkg.reduce_copy_ptrs(sp, dp, self.n, cfg["dt"], cfg["op"], cfg["arg"], None, False, self.handle)
            if per_launch or i == total - 1:
                ev[i][1].record(self.stream)

        with torch.cuda.device(self.dev):
            local_s, max_s = timed_steps(step, steps, warmup, lambda: torch.cuda.synchronize(self.dev), dist,
                                         self.dev)
        if per_launch:
            ms = [ev[warmup + i][0].elapsed_time(ev[warmup + i][1]) for i in range(steps)]
            kernel_s = sum(ms) / len(ms) / 1e3
        else:
            kernel_s = ev[warmup][0].elapsed_time(ev[total - 1][1]) / steps / 1e3
        self.last_set = (total - 1) % len(self.sets)
        return local_s, max_s, kernel_s

    def free(self):
        import torch
        self.sets = []
        torch.cuda.empty_cache()


def roofline(cfg, config_name: str, kernel_s: float, per_launch: bool = False) -> dict:
    achieved = algorithmic_bytes(cfg) / kernel_s / 1e9
    traffic, src = load_traffic(config_name)
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic, "kernel": KERNEL,
            "avg_kernel_us": round(kernel_s * 1e6, 2),
            "timing": ("HIP events around every launch on its stream" if per_launch else
                       "HIP events around the timed region on the launch stream / steps"),
            "traffic_source": src}


def load_traffic(config_name: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config_name}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def extra_configs(pkg, steps: int = 20, warmup: int = 5, names=EXTRA_ORDER) -> dict:
    """BASELINE configs[2] and [3] (C3 fp16/bf16 K=8 256 MiB, C4 int32/int8 min/max/prod K=4 64 MiB)
    after the headline's timed region, each on 3 rotating buffer sets: W untimed + S timed launches,
    average kernel time from HIP events on the launch stream."""
    out = {}
    for i, name in enumerate(names):
        cfg = CONFIGS[name]
        wl = DeviceWorkload(pkg, cfg, local_device_index(), seed=2000 + i)
        _, _, kernel_s = wl.run(steps, warmup, _Solo())
        exact = side_leg(wl.check_exact, wl.last_set)
        sets = side_leg(wl.per_set)
        wl.free()
        r = roofline(cfg, name, kernel_s)
        out[name] = {"workload": cfg["workload"], "dtype": cfg["dtype"], "bytes_per_launch": algorithmic_bytes(cfg),
                     "achieved": r["achieved"], "frac": r["frac"], "avg_kernel_us": r["avg_kernel_us"],
                     "traffic": r["traffic"], "traffic_source": r["traffic_source"], "steps": steps,
                     "warmup": warmup, "exact": exact.get("exact"), "exact_check": exact}
        out[name].update(sets if "error" not in sets else {"per_set_error": sets})
    return out


# ---- C1: the emulated ring all-reduce (BASELINE configs[0]) -------------------------------------
def c1_ring(iters: int = 20) -> dict:
    """BASELINE configs[0]: fp32 sum all-reduce of 4 MiB per rank over 2 emulated ranks, the ring
    schedule (runRing, src/device/all_reduce.h:12-84) with SIMPLE steps, restated in libnexr_ring.
    Three reduce-copy back ends under the same schedule: the HIP kernel on device-resident buffers,
    the HIP kernel behind host staging buffers (the fork's setting: NEX "device memory" is host
    memory), and the CPU oracle (every step on a host core, the reference's own path). Inputs are
    small integers, so every fold order gives the same fp32 sums and each result is checked exactly."""
    import ctypes
    import numpy as np
    import torch
    import oracle

    ring = importlib.import_module("nex-nccl_amd.ring")
    n, count = 2, 1 << 20
    rng = np.random.default_rng(1)
    x = [rng.integers(-1000, 1000, count).astype(np.float32) for _ in range(n)]
    expect = x[0] + x[1]
    ol = oracle.lib()
    cpu_fn = ctypes.cast(ol.oracle_reduce_copy_emulated_fn, ctypes.c_void_p).value
    out = {"workload": "fp32 sum all-reduce, 4 MiB per rank, 2 emulated ranks, ring SIMPLE, 1 channel"}
    legs = (("device", ring.DEVICE_MEMORY, None, ring.PROTO_SIMPLE),
            ("device_ll", ring.DEVICE_MEMORY, None, ring.PROTO_LL),
            ("device_ll128", ring.DEVICE_MEMORY, None, ring.PROTO_LL128),
            ("host_staged", ring.HOST_MEMORY, None, ring.PROTO_SIMPLE),
            ("host_registered", ring.HOST_MEMORY, None, ring.PROTO_SIMPLE),
            ("cpu_oracle", ring.HOST_MEMORY, cpu_fn, ring.PROTO_SIMPLE))
    nexr = importlib.import_module("nex-nccl_amd")
    for name, mode, fn, proto in legs:
        if mode == ring.DEVICE_MEMORY:  # rank r's buffers on rank r's GPU (libnexr_ring: r mod visible)
            devs = [torch.device("cuda", r % torch.cuda.device_count()) for r in range(n)]
            send = [torch.from_numpy(v).to(d) for v, d in zip(x, devs)]
            recv = [torch.zeros(count, dtype=torch.float32, device=d) for d in devs]
            for d in set(devs):
                torch.cuda.synchronize(d)
            out["device_gpus"] = [d.index for d in devs]
        else:
            send, recv = [v.copy() for v in x], [np.zeros(count, np.float32) for _ in range(n)]
        sp = [t.data_ptr() if hasattr(t, "data_ptr") else t.ctypes.data for t in send]
        rp = [t.data_ptr() if hasattr(t, "data_ptr") else t.ctypes.data for t in recv]
        reps = iters if fn is None else max(2, iters // 10)
        # host_registered: the integration INTEGRATION.md §2b recommends — the user buffers registered
        # once with nexrHostRegister (outside the timing), so every step is one zero-copy kernel whose
        # buffers are classified from the registration cache (the FIFOs come from nexrHostMemAlloc)
        handles = [nexr.host_register(a.ctypes.data, a.nbytes) for a in send + recv] if name == "host_registered" else []
        try:
            with ring.RingComm(n, mode, 0, fn, protocol=proto, timeout_ms=10000) as comm:
                wait = comm.step_wait()
                comm.all_reduce(sp, rp, count, 7, 0)
                nexr.host_path_stats(reset=True)
                t0 = time.perf_counter()
                for _ in range(reps):
                    comm.all_reduce(sp, rp, count, 7, 0)
                dt = (time.perf_counter() - t0) / reps
                hp = nexr.host_path_stats(reset=True)
                ll_mode = comm.queued()
        finally:
            for h in handles:
                nexr.host_deregister(h)
        got = [r.cpu().numpy() if hasattr(r, "cpu") else r for r in recv]
        out[name] = {"ms_per_call": round(dt * 1e3, 3), "algbw_gbs": round(count * 4 / dt / 1e9, 2), "calls": reps,
                     "exact": all(np.array_equal(g, expect) for g in got)}
        if mode == ring.HOST_MEMORY and fn is None and hp["calls"]:
            # per reduce-copy step (nexrGetHostPathStats, summed over both rank threads): where the
            # host time of nexrReduceCopyHost goes; wait includes the kernel's run over PCIe
            steps = hp["calls"]
            out[name]["per_step"] = {
                "steps_per_call": round(steps / reps, 2), "zero_copy_steps": hp["zeroCopyCalls"] / steps,
                "registered_hits": hp["registeredHits"], "pointer_queries": hp["pointerQueries"],
                **{f"{k}_us": round(hp[k + "Ns"] / steps / 1e3, 2) for k in ("classify", "copy", "launch", "wait")}}
        if mode == ring.DEVICE_MEMORY:
            out[name]["step_wait"] = wait  # "word" with both ranks on one GPU, "sync" across GPUs
        if proto == ring.PROTO_LL:
            # how the LL steps ran (nexrRingCommGetQueued): device runs / queued / host-sequenced
            out[name]["ll_steps"] = {2: "device runs", 1: "queued launches", 0: "host-sequenced"}.get(ll_mode, ll_mode)
    out["note"] = ("plumbing, not a roofline config (SURVEY §8(d) C1); device_ll / device_ll128 run the same ring "
                   "with the LL / LL128 protocol steps (SURVEY §8(f) #3) in place of SIMPLE; cpu_oracle runs the same schedule with the "
                   "reference's CPU execution of reduceCopy (oracle_reduce_copy_emulated_fn: 480 emulated threads, "
                   "Unroll 4) as its reduce-copy on host cores")
    return out


# ---- CPU baseline: the oracle (C restatement) on the benchmarked configuration ------------------
def usable_cores() -> tuple:
    """(threads to use, how that was decided): the CPUs this process may run on, capped by the
    cgroup's CPU quota when one is set (a GPU box shows the whole machine's CPUs but grants a share)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    return n, f"sched_getaffinity {aff} CPUs" + (f", cgroup cpu.max quota {quota} CPUs" if quota else "")


def cpu_sample(cfg, n: int, seed: int = 7):
    import numpy as np
    rng = np.random.default_rng(seed)
    store = {0: np.uint8, 1: np.uint8, 2: np.uint32, 3: np.uint32, 4: np.uint64, 5: np.uint64, 6: np.uint16,
             7: np.float32, 8: np.float64, 9: np.uint16}[cfg["dt"]]
    if cfg["dt"] == 7:
        srcs = [(rng.random(n, dtype=np.float32) * 2 - 1) for _ in range(cfg["k"])]
    else:
        srcs = [rng.integers(0, 256, n * ESZ[cfg["dt"]], dtype=np.uint8).view(store) for _ in range(cfg["k"])]
    dsts = [np.empty_like(srcs[0]) for _ in range(cfg["m"])]
    return srcs, dsts


# The reference's geometry for a ring step's reduceCopy in the fork's g++ build (oracle/nexr_oracle.c,
# oracle_reduce_copy_emulated_fn): 480 worker threads (prims_simple.h:614), Unroll 4 (device.h:1131-1134).
REF_EXECUTION = (480, 4)


def cpu_baseline(cfg, seconds: float = 10.0, threads: int = 1, sample=None, emulated=REF_EXECUTION):
    """The C oracle over the FULL configuration (every buffer at cfg['buf_bytes']) for about
    `seconds`: returns (GB/s of algorithmic bytes, calls, seconds). `emulated` = (threads, unroll)
    runs the reference's own CPU execution of reduceCopy (cooperative emulated threads one after
    another over reduceCopyPacks' hunk layout); None runs the plain element loop."""
    import oracle

    n = cfg["buf_bytes"] // ESZ[cfg["dt"]]
    srcs, dsts = sample if sample is not None else cpu_sample(cfg, n)
    kw = dict(dsts=dsts, threads=threads, emulated=emulated)
    oracle.reduce_copy(srcs, cfg["m"], cfg["dt"], cfg["op"], cfg["arg"], **kw)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.reduce_copy(srcs, cfg["m"], cfg["dt"], cfg["op"], cfg["arg"], **kw)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gbs = reps * algorithmic_bytes(cfg) / el / 1e9
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


def cpu_baseline_entry(cfg, seconds: float) -> dict:
    n = cfg["buf_bytes"] // ESZ[cfg["dt"]]
    sample = cpu_sample(cfg, n)
    gbs1, reps1, el1 = cpu_baseline(cfg, seconds, threads=1, sample=sample)
    nthreads, how = usable_cores()
    gbsN, repsN, elN = cpu_baseline(cfg, max(2.0, seconds / 4), threads=nthreads, sample=sample)
    lp1, lreps1, lel1 = cpu_baseline(cfg, max(2.0, seconds / 3), threads=1, sample=sample, emulated=None)
    lpN, lrepsN, lelN = cpu_baseline(cfg, max(1.0, seconds / 6), threads=nthreads, sample=sample, emulated=None)
    mib = cfg["buf_bytes"] >> 20
    w, u = REF_EXECUTION
    return {"value": round(gbs1, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"the full benchmarked call: {cfg['k']} x {mib} MiB in, {cfg['m']} x {mib} MiB out "
                      f"({cfg['workload']}), {reps1} calls in {el1:.1f} s on 1 thread of {cpu_model()}",
            "note": f"times oracle_reduce_copy_emulated (oracle/nexr_oracle.c): the reference's CPU execution of "
                    f"reduceCopy restated — {w} emulated threads (a ring step's workers) run one after another on "
                    f"one pthread, as the fork's emulator runs a launch's fibers, each over reduceCopyPacks' hunk "
                    f"layout with Unroll {u} and a memcpy per pack; the compiled reference reduceCopy ran at "
                    f"{REF_CPU_GBS_SURVEY} GB/s on one core of the survey's container (SURVEY §6)",
            "all_cores": {"value": round(gbsN, 3), "cores": nthreads, "cores_from": how,
                          "sample": f"{repsN} calls in {elN:.1f} s, one emulated launch per pthread on a "
                                    f"contiguous slice"},
            "element_loop": {"value": round(lp1, 3), "cores": 1, "all_cores_value": round(lpN, 3),
                             "all_cores": nthreads,
                             "sample": f"{lreps1} calls in {lel1:.1f} s on 1 thread, {lrepsN} calls in "
                                       f"{lelN:.1f} s on {nthreads}",
                             "note": "the same arithmetic as a plain per-element loop (oracle_reduce_copy): what "
                                     "a straightforward CPU implementation reaches, not the reference's path"}}


# ---- N > 1: the C5 summary ----------------------------------------------------------------------
def c5_summary(n_gpus: int, bytes_step: int, steps: int, agg_seconds: float, n1_seconds: float,
               solo_seconds: list) -> dict:
    """aggregate GB/s over all GPUs, the same-run N=1 leg on GPU 0, every GPU's own
    rate when it runs alone, and aggregate / (N x N=1) as measured in this run."""
    agg = n_gpus * bytes_step * steps / agg_seconds / 1e9
    n1 = bytes_step * steps / n1_seconds / 1e9
    solo = [bytes_step * steps / s / 1e9 for s in solo_seconds]
    return {"aggregate_gbs": round(agg, 2), "n1_same_run_gbs": round(n1, 2),
            "solo_gbs_per_gpu": [round(x, 1) for x in solo],
            "aggregate_over_n_times_n1": round(agg / (n_gpus * n1), 4),
            "note": "per-GPU chunks are independent (no collective); solo_gbs_per_gpu = each GPU timed alone"}


def per_gpu_summary(ranks, bytes_step: int, steps: int) -> dict:
    """Per-rank wall and kernel rates of an N > 1 run: `ranks[r] = [wall seconds, kernel seconds per
    launch]`. `value` stays the aggregate (N x bytes / max wall); this shows how even the ranks were."""
    wall = [bytes_step * steps / w / 1e9 for w, _ in ranks]
    kern = [bytes_step / k / 1e9 if k > 0 else 0.0 for _, k in ranks]
    return {"value": round(sum(wall) / len(wall), 2), "unit": "GB/s",
            "wall_gbs": [round(x, 1) for x in wall], "kernel_gbs": [round(x, 1) for x in kern],
            "min_wall_gbs": round(min(wall), 2), "max_wall_gbs": round(max(wall), 2)}


def base_line(cfg, n_gpus: int, steps: int, warmup: int, value: float, max_s: float, parallelism: str) -> dict:
    return {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": n_gpus,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(max_s / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": cfg["dtype"],
        "data": DATA,
        "config": {"workload": cfg["workload"], "k_inputs": cfg["k"], "m_outputs": cfg["m"],
                   "bytes_per_buffer": cfg["buf_bytes"], "bytes_per_step_per_gpu": algorithmic_bytes(cfg),
                   "parallelism": parallelism},
    }


def _bounded(cmd, timeout_s: float):
    """Run a probe in its own process group; on a timeout the whole group (the probe and the ring
    ranks it started) is killed. Returns its last JSON line or an error record, never raises."""
    import signal
    import subprocess
    try:
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
        try:
            out, err = p.communicate(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.communicate()
            return {"error": f"timeout after {timeout_s:.0f} s"}
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        if p.returncode == 0 and lines:
            return json.loads(lines[-1])
        return {"error": f"exit {p.returncode}", "stderr": err[-300:]}
    except Exception as e:  # noqa: BLE001 - reported, not raised
        return {"error": repr(e)[:300]}


XGMI_LINK_GBS = 153.0  # one xGMI link, one direction (MI355X_MICROARCH.md; 7 links per GPU)
# Wall-time budget of an N > 1 line: the driver's BENCH timeout is 600 s; the whole line
# (timed region, checks, solo legs, node-wide host rate, xGMI probe) is kept under TOTAL_CAP_S, and the
# probe gets what is left of it, at most XGMI_BUDGET_S.
TOTAL_CAP_S = 300.0
XGMI_BUDGET_S = 180.0
XGMI_MARGIN_S = 15.0
# The probe's parts, in order, with their own limits (seconds). The process rings run twice, once with
# every rank thread waiting for its steps by stream synchronisation (the cross-GPU default) and once
# by the completion word (NEXR_STEP_WAIT=word): a mismatch under "word" alone is a step-visibility
# fault, a mismatch under both a link or schedule fault.
XGMI_PARTS = (("peer_step", ["--peer-step"], 45.0, 2),
              ("ring_processes", ["--ring-only", "--step-wait", "sync"], 40.0, 2),
              ("ring_processes_word", ["--ring-only", "--step-wait", "word"], 40.0, 2),
              ("ring_processes_all_gpus", ["--ring-all", "{n}", "--step-wait", "sync"], 55.0, 3),
              ("ring_processes_all_gpus_word", ["--ring-all", "{n}", "--step-wait", "word"], 55.0, 3))


def probe_budget(elapsed_s: float) -> float:
    """Seconds the xGMI probe may take after `elapsed_s` of the line: never past TOTAL_CAP_S."""
    return max(0.0, min(XGMI_BUDGET_S, TOTAL_CAP_S - XGMI_MARGIN_S - elapsed_s))


def xgmi_link_rates(res: dict) -> dict:
    """Next to every exact check of the probe, the rate that crossed xGMI against the one-link bound:
    the peer step's remote read / write (one 256 MiB operand over the link per launch), and the ring
    all-reduces (each rank sends 2(n-1)/n of its bytes to its successor over one link: busbw)."""
    if not isinstance(res, dict):
        return res
    for key in ("remote_read", "remote_write"):
        v = res.get(key)
        if isinstance(v, dict) and "xgmi_GBps" in v:
            v["link_bound_GBps"] = XGMI_LINK_GBS
            v["frac_of_link"] = round(v["xgmi_GBps"] / XGMI_LINK_GBS, 4)
    for key in ("ring_processes", "ring_processes_word", "ring_processes_all_gpus", "ring_processes_all_gpus_word"):
        v = res.get(key)
        if not isinstance(v, dict) or "per_protocol_bytes" not in v:
            continue
        n = len(v.get("gpus", [])) or 2
        for proto in v["per_protocol_bytes"].values():
            for r in proto.values():
                if isinstance(r, dict) and "algbw_GBps" in r:
                    r["busbw_GBps"] = round(r["algbw_GBps"] * 2 * (n - 1) / n, 2)
                    r["frac_of_link"] = round(r["busbw_GBps"] / XGMI_LINK_GBS, 4)
    v = res.get("resident_ring")
    if isinstance(v, dict):
        for r in v.values():
            if isinstance(r, dict) and "busbw_GBps" in r:
                r["frac_of_link"] = round(r["busbw_GBps"] / XGMI_LINK_GBS, 4)
    res["link_bound_GBps"] = XGMI_LINK_GBS
    return res


def step_wait_verdict(res: dict) -> dict:
    """Both step waits side by side for each process ring that ran: exact on every rank under the
    synchronisation and under the completion word, and what a difference means."""
    out = {}
    for key in ("ring_processes", "ring_processes_all_gpus"):
        sync, word = res.get(key), res.get(key + "_word")
        if not isinstance(sync, dict) and not isinstance(word, dict):
            continue
        ex = lambda v: v.get("exact_all_ranks") if isinstance(v, dict) else None  # noqa: E731
        out[key] = {"sync_exact_all_ranks": ex(sync), "word_exact_all_ranks": ex(word),
                    "sync_in_effect": (sync or {}).get("step_wait_in_effect"),
                    "word_in_effect": (word or {}).get("step_wait_in_effect")}
    sync_ok = [v["sync_exact_all_ranks"] for v in out.values()]
    word_ok = [v["word_exact_all_ranks"] for v in out.values()]
    out["visibility_fault"] = any(s is True and w is False for s, w in zip(sync_ok, word_ok))
    out["link_or_schedule_fault"] = any(s is False for s in sync_ok)
    out["note"] = ("the cross-GPU default is the synchronisation (nexrRingCommGetStepWait); a ring exact under "
                   "sync but not under the word would be a step-visibility fault, not a link fault")
    return out


def xgmi_probe(budget_s: float = XGMI_BUDGET_S):
    """The peer-memory step over xGMI (tools/xgmi_probe.py), after the timed region, each part in a
    bounded subprocess of its own so one hang cannot cost the others or the line: GPU 0's kernel with
    an operand in GPU 1's HBM, the two-rank process ring under both step waits, and with three or more
    GPUs the process ring over all of them (up to 8) under both step waits. With NEXR_XGMI_RESIDENT=1
    and the opt-in extras library built, also the resident ring over all GPUs (beyond SURVEY §8). The
    parts share `budget_s`; a part that times out or finds the budget spent is recorded as such.
    Reported, never allowed to fail the bench line."""
    import torch
    probe = os.path.join(ROOT, "tools", "xgmi_probe.py")
    t0 = time.perf_counter()
    t_end = t0 + budget_s
    n_dev = torch.cuda.device_count()

    def part(args, limit):
        left = t_end - time.perf_counter()
        if left < 5:
            return {"error": "skipped: the probe budget is spent"}
        return _bounded([sys.executable, probe] + args, min(limit, left))

    res = None
    part_s = {}
    for key, args, limit, min_gpus in XGMI_PARTS:
        if n_dev < min_gpus:
            continue
        t = time.perf_counter()
        out = part([a.replace("{n}", str(min(n_dev, 8))) for a in args], limit)
        part_s[key] = round(time.perf_counter() - t, 1)
        if res is None:
            res = out
            if not isinstance(res, dict) or "skipped" in res:
                break
        else:
            res[key] = out
    if isinstance(res, dict) and "skipped" not in res and os.environ.get("NEXR_XGMI_RESIDENT") == "1":
        t = time.perf_counter()
        res["resident_ring"] = part(["--resident-only", str(min(n_dev, 8))], 60.0)
        part_s["resident_ring"] = round(time.perf_counter() - t, 1)
    if res is None:
        res = {"skipped": f"needs 2 GPUs, found {n_dev}"}
    if isinstance(res, dict) and "skipped" not in res:
        res["step_wait_modes"] = step_wait_verdict(res)
    if isinstance(res, dict):
        res["budget_s"] = round(budget_s, 1)
        res["part_s"] = part_s
        res["wall_s"] = round(time.perf_counter() - t0, 1)
    return xgmi_link_rates(res)


def h2d_inclusive(pkg, cfg, reps: int = 3):
    """Rate with the host<->device traffic included (nexrReduceCopyHost on host buffers).

    Pinned buffers take the zero-copy path (the kernel reads/writes host memory over PCIe, both
    directions at once); pageable buffers of a call this large go through the host copy team into
    pinned zero-copy slots (nexr_api.cpp reduceCopyHostTeam)."""
    import numpy as np
    import torch

    n = cfg["buf_bytes"] // ESZ[cfg["dt"]]

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
    split = side_leg(explicit_copies, pkg, cfg, pinned_s, pinned_d, reps)
    del pinned_s, pinned_d
    rng = np.random.default_rng(3)
    page_s = [rng.integers(0, 256, cfg["buf_bytes"], dtype=np.uint8) for _ in range(cfg["k"])]
    page_d = [np.empty(cfg["buf_bytes"], dtype=np.uint8) for _ in range(cfg["m"])]
    t_page = run(page_s, page_d)
    alg = algorithmic_bytes(cfg)
    return {"value": round(alg / t_pin / 1e9, 2), "unit": "GB/s", "ms_per_call": round(t_pin * 1e3, 3),
            "path": "nexrReduceCopyHost, pinned host buffers: zero-copy kernel over PCIe Gen5 x16",
            "explicit_copies": split,
            "pageable": {"value": round(alg / t_page / 1e9, 2), "ms_per_call": round(t_page * 1e3, 3),
                         "path": "host copy team (8 threads) into pinned zero-copy slots, 32 MiB chunks, "
                                 "kernel over PCIe, copy team out (the path for calls of 256 MiB or more; "
                                 "4-256 MiB: runtime H2D -> kernel -> D2H chunk pipeline; up to 4 MiB: the "
                                 "calling thread's copies into zero-copy slots)"}}


def explicit_copies(pkg, cfg, pinned_s, pinned_d, reps: int = 3) -> dict:
    """SURVEY §8(d)'s H<->D-inclusive measurement as stated: K H2D copies from pinned host buffers
    (hipMemcpyAsync), the kernel on the device copies, M D2H copies, one stream, timed end to end with
    HIP events between the phases, so the copy / kernel split is reported. The zero-copy path above
    (`value`) overlaps the two PCIe directions and is the faster way to run the same call."""
    import torch
    n = cfg["buf_bytes"] // ESZ[cfg["dt"]]
    dev = torch.device("cuda", local_device_index())
    stream = torch.cuda.current_stream(dev)
    d_s = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8, device=dev) for _ in pinned_s]
    d_d = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8, device=dev) for _ in pinned_d]
    sp, dp = [t.data_ptr() for t in d_s], [t.data_ptr() for t in d_d]
    phases = {"h2d": [], "kernel": [], "d2h": []}
    with torch.cuda.device(dev):
        for it in range(reps + 1):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record(stream)
            for d, h in zip(d_s, pinned_s):
                d.copy_(h, non_blocking=True)
            ev[1].record(stream)
            pkg.reduce_copy_ptrs(sp, dp, n, cfg["dt"], cfg["op"], cfg["arg"], None, False, stream.cuda_stream)
            ev[2].record(stream)
            for h, d in zip(pinned_d, d_d):
                h.copy_(d, non_blocking=True)
            ev[3].record(stream)
            ev[3].synchronize()
            if it:  # the first round warms the copy path
                for k, (a, b) in zip(("h2d", "kernel", "d2h"), zip(ev[:3], ev[1:])):
                    phases[k].append(a.elapsed_time(b))
    ms = {k: sum(v) / len(v) for k, v in phases.items()}
    total = sum(ms.values())
    return {"value": round(algorithmic_bytes(cfg) / (total / 1e3) / 1e9, 2), "unit": "GB/s",
            "ms_per_call": round(total, 3), "h2d_ms": round(ms["h2d"], 3), "kernel_ms": round(ms["kernel"], 4),
            "d2h_ms": round(ms["d2h"], 3),
            "h2d_gbs": round(cfg["k"] * cfg["buf_bytes"] / (ms["h2d"] / 1e3) / 1e9, 2),
            "d2h_gbs": round(cfg["m"] * cfg["buf_bytes"] / (ms["d2h"] / 1e3) / 1e9, 2),
            "path": f"{cfg['k']} hipMemcpyAsync H2D from pinned buffers -> nexrReduceCopy on device copies -> "
                    f"{cfg['m']} D2H, one stream, HIP events between the phases"}


def h2d_pinned_all_ranks(pkg, cfg, dist, device, reps: int = 3) -> dict:
    """N > 1: every rank's C2 call on its own pinned host buffers (the zero-copy path over its own
    PCIe link) at the same time, after a barrier — the host<->device-inclusive rate of the whole node,
    where host memory and the links are shared (NUMA placement of pinned buffers is the
    only coupling between GPUs, and only for this variant)."""
    import torch

    n = cfg["buf_bytes"] // ESZ[cfg["dt"]]
    err = None
    try:  # a rank that cannot pin its buffers still takes part in the barrier and the gather
        srcs = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8).pin_memory() for _ in range(cfg["k"])]
        dsts = [torch.empty(cfg["buf_bytes"], dtype=torch.uint8).pin_memory() for _ in range(cfg["m"])]
        for t in srcs:
            t.random_(0, 255)
        sp, dp = [t.data_ptr() for t in srcs], [t.data_ptr() for t in dsts]
        pkg.reduce_copy_ptrs(sp, dp, n, cfg["dt"], cfg["op"], cfg["arg"], None, False, 0, host=True)  # warm
    except Exception as e:  # noqa: BLE001 - reported in the line
        err = repr(e)[:200]
    dist.barrier()
    mine = -1.0
    if err is None:
        try:
            t0 = time.perf_counter()
            for _ in range(reps):
                pkg.reduce_copy_ptrs(sp, dp, n, cfg["dt"], cfg["op"], cfg["arg"], None, False, 0, host=True)
            mine = time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001
            err = repr(e)[:200]
    per = dist.gather([mine], device)
    srcs = dsts = None
    if any(p[0] <= 0 for p in per):
        return {"error": err or "another rank failed", "per_rank_s": [p[0] for p in per]}
    slowest = max(p[0] for p in per)
    alg = algorithmic_bytes(cfg)
    return {"value": round(dist.world * alg * reps / slowest / 1e9, 2), "unit": "GB/s",
            "per_rank_gbs": [round(alg * reps / p[0] / 1e9, 2) for p in per], "ms_per_call_max": round(slowest / reps * 1e3, 3),
            "path": "nexrReduceCopyHost on pinned host buffers (zero-copy over PCIe), every rank at once"}


def side_leg(fn, *a):
    """A leg measured after the headline's timed region (other configurations, C1, the CPU baseline,
    host-inclusive rates): a Python-level failure there is recorded in the line, never raised, so it
    cannot cost the headline. (C1's device ranks land on GPUs 0 and 1 on a multi-GPU node, a peer
    path the one-GPU boxes do not exercise.)"""
    try:
        return fn(*a)
    except Exception as e:  # noqa: BLE001 - any failure is reported in the line
        return {"error": repr(e)[:300], "leg": fn.__name__}


# ---- the two ways to drive N GPUs ---------------------------------------------------------------
class Phases:
    """Wall seconds of each phase of a line since the process started (`phase_s`), so a line whose run
    came close to the driver's timeout shows where the time went."""

    def __init__(self):
        self.t = time.perf_counter()
        self.s = {"startup": round(self.t - _T0, 2)}

    def mark(self, name: str) -> None:
        now = time.perf_counter()
        self.s[name] = round(now - self.t, 2)
        self.t = now

    def elapsed(self) -> float:
        return time.perf_counter() - _T0

    def summary(self) -> dict:
        return dict(self.s, total=round(self.elapsed(), 2), cap_s=TOTAL_CAP_S)


def main_ranks(args, cfg, pkg) -> dict | None:
    """One process per GPU (N=1 plain, or N>1 under torchrun): each rank times its own chunk."""
    import torch

    dist = Dist(os.environ.get("NEXR_BENCH_BACKEND", "gloo"))
    if dist.world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={dist.world}")
    dev_index = local_device_index()
    torch.cuda.set_device(dev_index)
    per_launch = args.events == "launch"
    ph = Phases()
    wl = DeviceWorkload(pkg, cfg, dev_index, seed=1000 + dist.rank)
    ph.mark("inputs")
    local_s, max_s, kernel_s = wl.run(args.steps, args.warmup, dist, per_launch)
    ph.mark("timed_region")
    bytes_step = algorithmic_bytes(cfg)
    value = dist.world * bytes_step * args.steps / max_s / 1e9
    ranks = dist.gather([local_s, kernel_s], wl.dev)
    # After the timed region: every rank checks its own last output bit-exactly against the oracle;
    # rank 0 also times each of its rotating sets.
    exact = side_leg(wl.check_exact, wl.last_set)
    exact_ranks = [f[0] == 1.0 for f in dist.gather([1.0 if exact.get("exact") is True else 0.0], wl.dev)]
    sets = side_leg(wl.per_set) if dist.rank == 0 else None
    ph.mark("exact_checks_and_per_set")
    c5 = None
    if dist.world > 1:
        # Same-run legs: rank 0's GPU alone (the N=1 reference), then every GPU alone in turn.
        solo = []
        for r in range(dist.world):
            dist.barrier()
            s = wl.run(args.steps, args.warmup, _Solo())[0] if dist.rank == r else 0.0
            solo.append(dist.max(s, wl.dev))
            dist.barrier()
        c5 = c5_summary(dist.world, bytes_step, args.steps, max_s, solo[0], solo)
        ph.mark("solo_legs")
    h2d_all = None
    if dist.world > 1 and not args.no_h2d:
        wl.free()
        h2d_all = h2d_pinned_all_ranks(pkg, cfg, dist, wl.dev)
        ph.mark("h2d_all_ranks")
    result = None
    if dist.rank == 0:
        result = base_line(cfg, dist.world, args.steps, args.warmup, value, max_s,
                           f"independent chunks x{dist.world} (no collective)" +
                           (f", one process per GPU ({dist.backend} barrier)" if dist.world > 1 else "") +
                           (f"; REHEARSAL: {dist.world} ranks folded onto {torch.cuda.device_count()} GPU(s)"
                            if torch.cuda.device_count() < dist.world else ""))
        result["roofline"] = roofline(cfg, args.config, kernel_s, per_launch)
        result["roofline"].update(sets if "error" not in sets else {"per_set_error": sets})
        result["exact"] = all(exact_ranks)
        result["exact_check"] = dict(exact, per_rank=exact_ranks)
        result["cpu_baseline"] = None
        result["h2d_inclusive"] = None
        if dist.world == 1:
            if not args.no_extra:
                wl.free()
                result["extra_configs"] = side_leg(extra_configs, pkg)
                result["c1_ring"] = side_leg(c1_ring)
            if not args.no_cpu:
                result["cpu_baseline"] = side_leg(cpu_baseline_entry, cfg, args.cpu_seconds)
            if not args.no_h2d:
                result["h2d_inclusive"] = side_leg(h2d_inclusive, pkg, cfg)
        else:
            result["per_gpu"] = per_gpu_summary(ranks, bytes_step, args.steps)
            result["c5"] = c5
            result["h2d_inclusive"] = h2d_all
            if not args.no_xgmi:
                result["xgmi_probe"] = xgmi_probe(probe_budget(ph.elapsed()))
                ph.mark("xgmi_probe")
            result["phase_s"] = ph.summary()
        print(json.dumps(result), flush=True)
    dist.barrier()
    dist.close()
    return result


def main_fanout(args, cfg, pkg) -> dict:
    """N>1 GPUs from ONE process, no launcher: nexrReduceCopyMultiDevice runs GPU d's chunk on a host
    thread of its own (hipSetDevice, its own stream, a shared start barrier, hipStreamSynchronize).
    The library reports the time from the barrier's release to the last GPU's completion."""
    import torch

    n_vis = torch.cuda.device_count()
    # NEXR_BENCH_FOLD=1 folds the N chunks onto the visible GPUs (chunk d on GPU d mod n): a rehearsal
    # of this path on a box with fewer GPUs; the line then says so in config.parallelism.
    fold = os.environ.get("NEXR_BENCH_FOLD") == "1"
    if n_vis < args.gpus and not fold:
        raise SystemExit(f"--gpus {args.gpus} but only {n_vis} visible GPU(s)")
    devices = [d % n_vis for d in range(args.gpus)]
    ph = Phases()
    # Three rotating buffer sets per GPU, as the N=1 line: launch k of a GPU runs set k mod 3
    # (nexrReduceCopyMultiDeviceSets), so no launch re-reads the previous one's cache-resident bytes.
    wls = [DeviceWorkload(pkg, cfg, dev, seed=1000 + d, sets=FANOUT_SETS) for d, dev in enumerate(devices)]
    for d in sorted(set(devices)):
        torch.cuda.synchronize(d)
    works = [[wl.work(s) for s in range(FANOUT_SETS)] for wl in wls]
    bytes_step = algorithmic_bytes(cfg)
    ph.mark("inputs")

    def timed(ws, ds):
        pkg.reduce_copy_multi_device_sets(ws, ds, cfg["dt"], cfg["op"], reps=max(1, args.warmup))
        return pkg.reduce_copy_multi_device_sets(ws, ds, cfg["dt"], cfg["op"], reps=args.steps)

    agg_s = timed(works, devices)
    ph.mark("timed_region")
    solo = [timed([works[i]], [devices[i]]) for i in range(args.gpus)]
    ph.mark("solo_legs")
    value = args.gpus * bytes_step * args.steps / agg_s / 1e9
    result = base_line(cfg, args.gpus, args.steps, args.warmup, value, agg_s,
                       f"independent chunks x{args.gpus} (no collective), one process, "
                       f"nexrReduceCopyMultiDeviceSets (a host thread + stream per GPU, {FANOUT_SETS} rotating sets)" +
                       (f"; REHEARSAL: {args.gpus} chunks folded onto {n_vis} GPU(s)" if n_vis < args.gpus else ""))
    # Every GPU's output against the oracle (outside the timed legs; each set holds its last output).
    checks = [side_leg(wl.check_exact, 0) for wl in wls]
    result["exact"] = all(c.get("exact") is True for c in checks)
    result["exact_check"] = {"per_gpu": [c.get("exact") for c in checks],
                             "checked_elements_per_gpu": checks[0].get("checked_elements"),
                             "check": checks[0].get("check", checks[0].get("error"))}
    ph.mark("exact_checks")
    # Roofline of the kernel itself: HIP events on GPU 0's launch stream, 3 rotating sets.
    for wl in wls:
        wl.free()
    wl0 = DeviceWorkload(pkg, cfg, 0, seed=1000)
    _, _, kernel_s = wl0.run(args.steps, args.warmup, _Solo())
    sets = side_leg(wl0.per_set)
    wl0.free()
    result["roofline"] = roofline(cfg, args.config, kernel_s)
    result["roofline"].update(sets if "error" not in sets else {"per_set_error": sets})
    result["cpu_baseline"] = None
    result["h2d_inclusive"] = None
    result["c5"] = c5_summary(args.gpus, bytes_step, args.steps, agg_s, solo[0], solo)
    result["c5"]["timing"] = ("nexrReduceCopyMultiDeviceSets: barrier release to the last GPU's completion, "
                              f"{FANOUT_SETS} rotating buffer sets per GPU (as the N=1 line)")
    result["c5"]["sets_per_gpu"] = FANOUT_SETS
    ph.mark("roofline_legs")
    if not args.no_xgmi:
        result["xgmi_probe"] = xgmi_probe(probe_budget(ph.elapsed()))
        ph.mark("xgmi_probe")
    result["phase_s"] = ph.summary()
    print(json.dumps(result), flush=True)
    return result


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-h2d", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3/C4 extra configurations (N=1 only)")
    ap.add_argument("--no-xgmi", action="store_true", help="skip the xGMI peer-step probe (N > 1 only)")
    ap.add_argument("--events", choices=["launch", "region"], default="region",
                    help="HIP events around every launch, or only around the timed region (default)")
    args = ap.parse_args(argv)
    if args.config != "c2":
        args.no_extra = True  # the extras are measured beside the headline configuration only

    pkg = importlib.import_module("nex-nccl_amd")
    pkg.lib()
    cfg = CONFIGS[args.config]
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        return main_fanout(args, cfg, pkg)
    return main_ranks(args, cfg, pkg)


if __name__ == "__main__":
    main()
