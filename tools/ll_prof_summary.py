#!/usr/bin/env python3
"""Kernel durations of a `rocprofv3 --kernel-trace` run of tools/ll_rate.py, matched launch for launch
to the lines ll_rate printed: per (data bytes, shape, protocol) the median kernel time over the timed
launches and its fraction of the 8 TB/s HBM peak for the algorithmic bytes ll_rate states.

    python3 tools/ll_prof_summary.py --trace <ll_kernel_trace.csv> --rate <ll_rate.jsonl> [--out FILE]

ll_rate's launch order per size: one LL and one LL128 send step that fill the recv wires, then for
each shape, per protocol (ll, ll128, simple), 3 warm-up launches and 7 blocks of `reps` launches."""
import argparse
import csv
import json
import statistics

PEAK_GBS = 8000.0


def nexr_launches(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "nexr::" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--rate", required=True)
    ap.add_argument("--out")
    a = ap.parse_args(argv)
    launches = nexr_launches(a.trace)
    lines = [json.loads(x) for x in open(a.rate) if x.startswith("{")]
    i, size, out = 0, None, []
    for ln in lines:
        if ln["data_bytes"] != size:  # the two wire-filling steps
            size = ln["data_bytes"]
            i += 2
        for proto in ("ll", "ll128", "simple"):
            n = 3 + 7 * ln["reps"]
            seg = launches[i:i + n]
            i += n
            names = {s[2].split("<")[0] for s in seg}
            want = {"ll": "reduce_copy_ll_kernel", "ll128": "reduce_copy_ll128_kernel", "simple": "reduce_copy_kernel"}
            assert len(seg) == n and all(want[proto] in nm for nm in names), (ln["shape"], proto, names)
            us = statistics.median((e - s) / 1e3 for s, e, _ in seg[3:])
            alg = ln[proto]["alg_bytes"]
            out.append({"data_bytes": size, "shape": ln["shape"], "proto": proto, "kernel_us": round(us, 2),
                        "GBps": round(alg / us / 1e3, 1), "frac": round(alg / us / 1e3 / PEAK_GBS, 3),
                        "event_us": ln[proto]["us"]})
    assert i == len(launches), f"{len(launches) - i} launches left over"
    text = ["data_bytes shape               proto   kernel_us    GB/s   frac  (event us/launch)"]
    for r in out:
        text.append(f"{r['data_bytes']:>10} {r['shape']:<20} {r['proto']:<6} {r['kernel_us']:>9} {r['GBps']:>8} "
                    f"{r['frac']:>6}  ({r['event_us']})")
    body = "\n".join(text)
    print(body)
    if a.out:
        with open(a.out, "w") as f:
            f.write(body + "\n")
    return out


if __name__ == "__main__":
    main()
