#!/usr/bin/env python3
"""Long random parity sweep of nexrReduceCopy against the C oracle (test infrastructure: the oracle
is the checker, the ABI the thing checked). The GPU suite's fuzz (tests/test_reduce_copy_gpu.py::
test_random_fuzz_against_oracle) runs 300 cases of up to 300,001 elements; this runs as many cases as
fit in `--seconds`, with sizes up to `--max-mib` per buffer drawn log-uniformly so the three cache
policies (plain < 64 MiB streamed <= nt loads < 512 MiB <= nt loads + stores) and their geometries are
all reached, every datatype x op (sum, prod, min, max, premulsum, sumpostdiv) x K 1-8 x M 1-8, shared
and mixed 16-B phases, guard bytes around every output, and ~1 in 8 cases in place (dst0 = src0).

    python tools/fuzz_long.py --seconds 240 --seed 1 > gpurun_out/fuzz.jsonl

Prints a progress line every 20 cases on stderr, one JSON line per failing case and a summary line;
exits 1 on any mismatch."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402
import oracle  # noqa: E402
import test_reduce_copy_gpu as rc  # noqa: E402  (run_gpu, same, _case_args)

nexr = __import__("importlib").import_module("nex-nccl_amd")

OPS = [("sum", mg.SUM), ("prod", mg.PROD), ("min", mg.MINMAX), ("max", mg.MINMAX), ("premulsum", mg.PREMULSUM),
       ("sumpostdiv", mg.SUMPOSTDIV)]


def one_case(rng, case, max_bytes, budget_bytes):
    dt = int(rng.choice(sorted(mg.DT_NAMES)))
    name, op = OPS[int(rng.integers(0, len(OPS)))]
    if name == "sumpostdiv" and dt not in mg.INTS:
        name, op = "sum", mg.SUM
    k = int(rng.integers(1, 9))
    m = int(rng.integers(1, 9))
    esz = np.dtype(mg.STORE[dt]).itemsize
    # log-uniform bytes per buffer in [1 element, max_bytes], capped so (K + M) buffers fit the budget
    cap = max(esz, min(max_bytes, budget_bytes // (k + m)))
    nbytes = int(np.exp(rng.uniform(np.log(esz), np.log(cap))))
    n = max(1, nbytes // esz + int(rng.integers(-3, 4)))
    mode = int(rng.integers(0, 3))
    if mode == 0:
        so, do = [0] * k, [0] * m
    elif mode == 1:
        ph = int(rng.integers(0, 16 // esz)) * esz
        so, do = [ph] * k, [ph] * m
    else:
        so = [int(rng.integers(0, 16)) for _ in range(k)]
        do = [int(rng.integers(0, 16)) for _ in range(m)]
    arg, pre, post = rc._case_args(dt, name, op, k, rng)
    srcs = mg.gen_inputs(dt, k, n, 70000 + case, special=True)
    exp = oracle.reduce_copy(srcs, 1, dt, op, arg, pre, post, threads=16)[0]
    desc = {"case": case, "dt": mg.DT_NAMES[dt], "op": name, "k": k, "m": m, "n": n, "src_off": so, "dst_off": do}
    in_place = rng.integers(0, 8) == 0 and so[0] == do[0]
    if in_place:  # dst0 aliases src0 (NCCL's in-place all-reduce); the other dsts as usual
        desc["in_place"] = True
        sbufs = [rc._to_dev(s, o) for s, o in zip(srcs, so)]
        dbufs = [torch.full((n * esz + o + 64,), 0x5A, dtype=torch.uint8, device="cuda") for o in do[1:]]
        dp = [sbufs[0].data_ptr() + so[0]] + [b.data_ptr() + o for b, o in zip(dbufs, do[1:])]
        nexr.reduce_copy_ptrs([b.data_ptr() + o for b, o in zip(sbufs, so)], dp, n, dt, op, arg, pre, post,
                              torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs = [sbufs[0].cpu().numpy()[so[0]:so[0] + n * esz].view(mg.STORE[dt])]
        for b, o in zip(dbufs, do[1:]):
            host = b.cpu().numpy()
            if not ((host[:o] == 0x5A).all() and (host[o + n * esz:] == 0x5A).all()):
                return desc, False, "write outside the destination"
            outs.append(host[o:o + n * esz].view(mg.STORE[dt]))
    else:
        try:
            outs = rc.run_gpu(nexr, srcs, m, dt, op, arg, pre, post, src_off=so, dst_off=do)
        except AssertionError as e:
            return desc, False, str(e)
    ok = all(rc.same(dt, o, exp) for o in outs)
    return desc, ok, None if ok else "mismatch vs oracle"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-mib", type=float, default=160.0, help="largest buffer (MiB)")
    ap.add_argument("--budget-mib", type=float, default=1200.0, help="cap on (K + M) x buffer bytes")
    a = ap.parse_args()
    assert torch.cuda.is_available()
    rng = np.random.default_rng(a.seed)
    t_end = time.time() + a.seconds
    stats = {"cases": 0, "failed": 0, "bytes_checked": 0, "by_policy": {"plain": 0, "nt_load": 0, "nt_load_store": 0},
             "in_place": 0, "max_buffer_bytes": 0}
    case = 0
    while time.time() < t_end:
        desc, ok, why = one_case(rng, case, int(a.max_mib * (1 << 20)), int(a.budget_mib * (1 << 20)))
        esz = np.dtype(mg.STORE[[d for d, v in mg.DT_NAMES.items() if v == desc["dt"]][0]]).itemsize
        streamed = (desc["k"] + desc["m"]) * desc["n"] * esz
        pol = "plain" if streamed < 64 << 20 else ("nt_load" if streamed < 512 << 20 else "nt_load_store")
        stats["by_policy"][pol] += 1
        stats["cases"] += 1
        stats["bytes_checked"] += desc["m"] * desc["n"] * esz
        stats["in_place"] += int(desc.get("in_place", False))
        stats["max_buffer_bytes"] = max(stats["max_buffer_bytes"], desc["n"] * esz)
        if not ok:
            stats["failed"] += 1
            print(json.dumps(dict(desc, error=why)), flush=True)
        case += 1
        if case % 20 == 0:
            print(f"[fuzz] {case} cases, {stats['failed']} failed, {time.time() - t_end + a.seconds:.0f} s",
                  file=sys.stderr, flush=True)
        torch.cuda.empty_cache()
    stats["seed"] = a.seed
    stats["checker"] = "oracle/nexr_oracle.c (bit-exact; float NaNs by class as in tests/)"
    print(json.dumps(stats), flush=True)
    return 1 if stats["failed"] else 0


if __name__ == "__main__":
    sys.exit(main())
