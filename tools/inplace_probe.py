#!/usr/bin/env python3
"""Out-of-place vs in-place (dst == src0) reduce-copy at the C2 / C3 / C4 shapes, same algorithmic
bytes (K reads + 1 write), 3 rotating buffer sets, HIP events around 20 launches after 5 warm-up.
In place, the write stream lands on the rows src0 was just read from: one stream fewer open at the
DRAM. Tuning harness, not a test (in-place correctness is tests/test_reduce_copy_gpu.py)."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

nexr = importlib.import_module("nex-nccl_amd")
nexr.lib()
CASES = [("c2 f32 sum K=2", torch.float32, 2, 256 << 20), ("c3 bf16 sum K=8", torch.bfloat16, 8, 256 << 20),
         ("c3 f16 sum K=8", torch.float16, 8, 256 << 20), ("c4 i32 sum K=4", torch.int32, 4, 64 << 20)]
stream = torch.cuda.current_stream()
for name, dt, k, buf in CASES:
    n = buf // torch.empty((), dtype=dt).element_size()
    sets = []
    for _ in range(3):
        srcs = [(torch.rand(n, device="cuda") * 2 - 1).to(dt) if dt.is_floating_point else
                torch.randint(-1000, 1000, (n,), dtype=dt, device="cuda") for _ in range(k)]
        sets.append((srcs, torch.empty_like(srcs[0])))
    res = {}
    for mode in ("out_of_place", "in_place", "out_of_place", "in_place"):
        def launch(i):
            srcs, out = sets[i % 3]
            dst = srcs[0] if mode == "in_place" else out
            nexr.reduce_copy(srcs, [dst], nexr.DevRedOp.Sum, stream=stream)
        for i in range(5):
            launch(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(20):
            launch(5 + i)
        e1.record(stream)
        e1.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        res.setdefault(mode, []).append(round((k + 1) * buf / us / 1e3, 1))
    print(json.dumps({"case": name, "GBps": res}), flush=True)
    del sets
    torch.cuda.empty_cache()
