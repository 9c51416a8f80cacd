"""The 8-bit fold's cost at C4 over every committed measurement (VERDICT r03 "next" #3).

`kernel_over_u32_sum` = a C4 kernel's time over a uint32 sum of the same bytes on the same buffers.
int32 min/max/prod fold with one 32-bit instruction per dword per step, like the uint32 sum (prod's
v_mul_lo_u32 excepted), so the int32 ratio of the same op in the same line is the measurement's own
floor on that box; the int8 ratio minus it is the 8-bit fold's cost. Reads the bench lines' extra
configs and the production rows of the two same-box A/B files; writes the table to stdout.

    python tools/fold8_cost_stats.py > profiles/r04e_fold8_cost_stats.txt
"""
import json
import os
import re
import statistics as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = ["profiles/r03u_evidence_bench.json", "profiles/r03zc_bench.json", "profiles/r04b_bench.json",
         "profiles/r04d_evidence_bench.json"]
AB = {"profiles/r04a_fold8_ab.txt": "production U2 B512", "profiles/r04b_pack_order_ab_not_kept.txt": "production (PM=0)"}
OPS = ["min", "max", "prod"]


def from_line(path):
    d = json.load(open(os.path.join(ROOT, path)))
    ec = d.get("extra_configs", {})
    return {(t, op): ec[f"c4_{t}_{op}"]["kernel_over_u32_sum"] for t in ("i8", "i32") for op in OPS
            if f"c4_{t}_{op}" in ec}


def from_ab(path, row):
    out, cur = {}, None
    for ln in open(os.path.join(ROOT, path)):
        if not ln[:1].isspace():  # a configuration's header line
            m = re.match(r"^(?:C4 )?(int8|int32) (min|max|prod)", ln)
            cur = ("i8" if m.group(1) == "int8" else "i32", m.group(2)) if m else None
        elif cur and ln.strip().startswith(row):
            out[cur] = float(re.search(r"over u32(?: sum)? ([0-9.]+)", ln).group(1))
    return out


def main():
    sources = [(p, from_line(p)) for p in LINES] + [(p, from_ab(p, r)) for p, r in AB.items()]
    print("C4 K = 4, 64 MiB: kernel time over a uint32 sum of the same bytes on the same buffers\n")
    print(f"{'source':48s} " + " ".join(f"{t}_{op:>4s}" for t in ("i8", "i32") for op in OPS))
    diffs = {op: [] for op in OPS}
    i8 = {op: [] for op in OPS}
    i32 = {op: [] for op in OPS}
    for p, r in sources:
        if len(r) != 6:
            print(f"{p:48s} (incomplete: {sorted(r)})")
            continue
        print(f"{p:48s} " + " ".join(f"{r[(t, op)]:8.4f}" for t in ("i8", "i32") for op in OPS))
        for op in OPS:
            i8[op].append(r[("i8", op)])
            i32[op].append(r[("i32", op)])
            diffs[op].append(r[("i8", op)] - r[("i32", op)])
    n = len(diffs["min"])
    print(f"\n{n} same-box measurements; mean (sample sd) of each ratio, and of int8 minus int32 of the same op in the same measurement")
    allv = []
    for op in OPS:
        allv += diffs[op]
        print(f"  {op:4s}  int8 {st.mean(i8[op]):.4f} ({st.stdev(i8[op]):.4f})  int32 {st.mean(i32[op]):.4f} "
              f"({st.stdev(i32[op]):.4f})  int8 - int32 {st.mean(diffs[op]):+.4f} ({st.stdev(diffs[op]):.4f}, "
              f"se {st.stdev(diffs[op]) / n ** 0.5:.4f})")
    print(f"  all three ops: int8 - int32 {st.mean(allv):+.4f} (sd {st.stdev(allv):.4f}, se {st.stdev(allv) / len(allv) ** 0.5:.4f}, "
          f"n = {len(allv)})")


if __name__ == "__main__":
    main()
