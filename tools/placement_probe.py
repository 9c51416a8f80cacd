#!/usr/bin/env python3
"""Buffer placement vs reduce-copy rate (one rotating set of the bench ran C3 at
0.81-0.83 of peak, the other two at 0.75-0.77, same kernel, same bytes).

Times the production kernel (nexrReduceCopy through the ABI) with per-launch HIP events over
buffer sets placed three ways, launches interleaved round-robin so no launch follows one on its
own buffers:
  torch   separate torch allocations per buffer, as bench.py makes them (addresses logged);
  slab    one allocation per set, buffer s at base + s * (buf + delta) for chosen deltas: the
          relative offset of the K + M streams controlled by hand;
  perm    one slab, the destination placed at different positions among the sources.
Tuning harness, not a test: every output of every set is compared with the first set's output of
identical data at the end (identical inputs are written to every set)."""
import argparse
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

nexr = importlib.import_module("nex-nccl_amd")
nexr.lib()

CFG = {"c2": (torch.float32, 7, 2, 256 << 20), "c3_bf16": (torch.bfloat16, 9, 8, 256 << 20),
       "c3_f16": (torch.float16, 6, 8, 256 << 20), "c4_i32": (torch.int32, 2, 4, 64 << 20)}
MIB = 1 << 20


def fill(ref, bufs):
    for r, b in zip(ref, bufs):
        b.copy_(r)


def make_ref(dt, k, n, seed=5):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    if dt.is_floating_point:
        return [(torch.rand(n, device="cuda", generator=g) * 2 - 1).to(dt) for _ in range(k)]
    return [torch.randint(-1000, 1000, (n,), dtype=dt, device="cuda", generator=g) for _ in range(k)]


def slab_set(dt, k, n, buf, delta, order=None):
    """One allocation; buffer j (j < k: sources, j == k: destination, or as `order` permutes) at
    base + j * (buf + delta)."""
    stride = buf + delta
    esz = torch.empty((), dtype=dt).element_size()
    slab = torch.empty((k + 1) * stride + 4096, dtype=torch.uint8, device="cuda")
    base = (slab.data_ptr() + 4095) // 4096 * 4096 - slab.data_ptr()
    views = [slab[base + j * stride: base + j * stride + buf].view(dt) for j in range(k + 1)]
    order = order or list(range(k + 1))
    bufs = [views[j] for j in order]
    assert all(v.numel() == n for v in bufs) and esz * n == buf
    return slab, bufs[:k], bufs[k]


def rel(p, base):
    d = p - base
    return {"off_mib": round(d / MIB, 3), "mod_2m": d % (2 * MIB), "mod_64k": d % 65536}


def run_cases(name, cases, rounds, dtid):
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    times = {c["label"]: [] for c in cases}
    for _ in range(2):  # warm
        for c in cases:
            nexr.reduce_copy_ptrs(c["sp"], c["dp"], c["n"], dtid, 0, 0, None, False, h)
    for r in range(rounds):
        order = cases if r % 2 == 0 else list(reversed(cases))
        evs = []
        for c in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            nexr.reduce_copy_ptrs(c["sp"], c["dp"], c["n"], dtid, 0, 0, None, False, h)
            e1.record(stream)
            evs.append((c["label"], e0, e1))
        torch.cuda.synchronize()
        for lab, e0, e1 in evs:
            times[lab].append(e0.elapsed_time(e1) * 1e3)
    return times


def report(name, cases, times, bytes_per_launch, kind):
    for c in cases:
        t = times[c["label"]]
        med = statistics.median(t)
        rec = {"probe": name, "kind": kind, "case": c["label"], "median_us": round(med, 2), "min_us": round(min(t), 2),
               "max_us": round(max(t), 2), "frac": round(bytes_per_launch / med / 1e3 / 8000, 4),
               "addrs": c.get("addrs")}
        print(json.dumps(rec), flush=True)


def hybrids(name, tsets, times, k, n, dtid, bpl, rounds):
    """Which buffers make a set fast or slow: the fastest and slowest torch sets, and sets built from
    the fast set's sources with the slow set's destination (and the reverse), half of each set's
    sources swapped, and each single source of the fast set swapped for the slow set's."""
    med = {c["label"]: statistics.median(times[c["label"]]) for c in tsets}
    fast = min(tsets, key=lambda c: med[c["label"]])
    slow = max(tsets, key=lambda c: med[c["label"]])
    h = k // 2
    mk = lambda lab, sp, dp: {"label": lab, "sp": sp, "dp": dp, "n": n}  # noqa: E731
    cases = [mk("fast", fast["sp"], fast["dp"]), mk("slow", slow["sp"], slow["dp"]),
             mk("fast_srcs_slow_dst", fast["sp"], slow["dp"]), mk("slow_srcs_fast_dst", slow["sp"], fast["dp"]),
             mk("fast_first_half_srcs", fast["sp"][:h] + slow["sp"][h:], fast["dp"]),
             mk("fast_second_half_srcs", slow["sp"][:h] + fast["sp"][h:], fast["dp"])]
    for j in range(k):
        sp = list(fast["sp"])
        sp[j] = slow["sp"][j]
        cases.append(mk(f"fast_with_slow_src{j}", sp, fast["dp"]))
    t = run_cases(name, cases, rounds, dtid)
    print(json.dumps({"probe": name, "kind": "hybrid_sets", "fast": fast["label"], "slow": slow["label"]}), flush=True)
    report(name, cases, t, bpl, "hybrid")


def per_buffer(name, tsets, n, dt, dtid, esz, rounds):
    """Every buffer of the torch sets alone: a K = 1 copy from it into one fixed scratch buffer, and
    a copy from a fixed source into it — a buffer whose own placement is slow shows here."""
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    scratch = torch.empty(n, dtype=dt, device="cuda")
    fixed = torch.empty(n, dtype=dt, device="cuda")
    fixed.zero_()
    bufs = []
    for c in tsets:
        for j, p in enumerate(c["sp"] + c["dp"]):
            bufs.append((f"{c['label']}.{j}", p))
    res = {lab: {"read": [], "write": []} for lab, _ in bufs}
    for _ in range(max(3, rounds // 3)):
        evs = []
        for lab, p in bufs:
            for kind, sp, dp in (("read", [p], [scratch.data_ptr()]), ("write", [fixed.data_ptr()], [p])):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                nexr.reduce_copy_ptrs(sp, dp, n, dtid, 0, 0, None, False, h)
                e1.record(stream)
                evs.append((lab, kind, e0, e1))
        torch.cuda.synchronize()
        for lab, kind, e0, e1 in evs:
            res[lab][kind].append(e0.elapsed_time(e1) * 1e3)
    for lab, _ in bufs:
        r = res[lab]
        print(json.dumps({"probe": name, "kind": "per_buffer_copy", "buffer": lab,
                          "copy_from_us": round(statistics.median(r["read"]), 2),
                          "copy_into_us": round(statistics.median(r["write"]), 2)}), flush=True)
    del scratch, fixed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3_bf16,c2")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--torch-sets", type=int, default=6)
    ap.add_argument("--deltas", default="0,4096,65536,1048576,2097152,2162688,4194304,16777216,134217728")
    args = ap.parse_args()
    deltas = [int(x) for x in args.deltas.split(",") if x]
    for name in args.configs.split(","):
        dt, dtid, k, buf = CFG[name]
        esz = torch.empty((), dtype=dt).element_size()
        n = buf // esz
        bpl = (k + 1) * buf
        ref = make_ref(dt, k, n)
        keep, cases = [], []
        # torch: separate allocations, as bench.py's DeviceWorkload
        for s in range(args.torch_sets):
            srcs = [torch.empty(n, dtype=dt, device="cuda") for _ in range(k)]
            dst = torch.empty(n, dtype=dt, device="cuda")
            fill(ref, srcs)
            keep.append((srcs, dst))
            ptrs = [t.data_ptr() for t in srcs] + [dst.data_ptr()]
            cases.append({"label": f"torch{s}", "sp": ptrs[:k], "dp": ptrs[k:], "n": n, "dst": dst,
                          "addrs": {"base_hex": hex(min(ptrs)),
                                    "bufs": [rel(p, min(ptrs)) for p in ptrs]}})
        # slab: controlled relative offsets
        for d in deltas:
            slab, srcs, dst = slab_set(dt, k, n, buf, d)
            fill(ref, srcs)
            keep.append(slab)
            cases.append({"label": f"slab_delta{d}", "sp": [t.data_ptr() for t in srcs], "dp": [dst.data_ptr()],
                          "n": n, "dst": dst, "addrs": {"base_hex": hex(srcs[0].data_ptr()), "delta": d}})
        # perm: destination first / middle / last in one slab (delta 0)
        for pos in (0, k // 2):
            order = [j for j in range(k + 1) if j != pos] + [pos]
            slab, srcs, dst = slab_set(dt, k, n, buf, 0, order)
            fill(ref, srcs)
            keep.append(slab)
            cases.append({"label": f"perm_dst_at{pos}", "sp": [t.data_ptr() for t in srcs], "dp": [dst.data_ptr()],
                          "n": n, "dst": dst, "addrs": {"dst_slot": pos}})
        torch.cuda.synchronize()
        times = run_cases(name, cases, args.rounds, dtid)
        report(name, cases, times, bpl, "rate")
        hybrids(name, cases[:args.torch_sets], times, k, n, dtid, bpl, args.rounds)
        per_buffer(name, cases[:args.torch_sets], n, dt, dtid, esz, args.rounds)
        first = cases[0]["dst"]
        same = all(torch.equal(c["dst"], first) for c in cases[1:])
        print(json.dumps({"probe": name, "all_outputs_identical": bool(same)}), flush=True)
        del keep, cases, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
