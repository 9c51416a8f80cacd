#!/usr/bin/env python3
"""Kernel durations of a `rocprofv3 --kernel-trace` run of tools/ll_rate.py, matched launch for launch
to the lines ll_rate printed: per (data bytes, shape, protocol) the median kernel time over the timed
launches and its fraction of the 8 TB/s HBM peak for the algorithmic bytes ll_rate states.

    python3 tools/ll_prof_summary.py --trace <ll_kernel_trace.csv> --rate <ll_rate.jsonl> [--out FILE]
    python3 tools/ll_prof_summary.py --fetch <FETCH_SIZE collection.csv> --write <WRITE_SIZE collection.csv> \
        --rate <ll_rate.jsonl> [--out FILE]          (HBM bytes per launch against the algorithmic bytes)

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


def nexr_counters(path, counter):
    """(dispatch id, value, kernel name) of every nexr dispatch in a --pmc counter collection."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "nexr::" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def segments(launches, lines):
    """Walk ll_rate's launch order: yields (line, proto, the timed launches of that leg)."""
    want = {"ll": "reduce_copy_ll_kernel", "ll128": "reduce_copy_ll128_kernel", "simple": "reduce_copy_kernel"}
    i, size = 0, None
    for ln in lines:
        if ln["data_bytes"] != size:  # the two wire-filling steps
            size = ln["data_bytes"]
            i += 2
        for proto in ("ll", "ll128", "simple"):
            n = 3 + 7 * ln["reps"]
            seg = launches[i:i + n]
            i += n
            names = {s[2].split("<")[0] for s in seg}
            assert len(seg) == n and all(want[proto] in nm for nm in names), (ln["shape"], proto, names)
            yield ln, proto, seg[3:]
    assert i == len(launches), f"{len(launches) - i} launches left over"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", help="kernel trace: durations")
    ap.add_argument("--fetch", help="--pmc FETCH_SIZE counter collection (with --write: HBM bytes)")
    ap.add_argument("--write", help="--pmc WRITE_SIZE counter collection")
    ap.add_argument("--rate", required=True)
    ap.add_argument("--out")
    a = ap.parse_args(argv)
    lines = [json.loads(x) for x in open(a.rate) if x.startswith("{")]
    out = []
    if a.trace:
        for ln, proto, seg in segments(nexr_launches(a.trace), lines):
            us = statistics.median((e - s) / 1e3 for s, e, _ in seg)
            alg = ln[proto]["alg_bytes"]
            out.append({"data_bytes": ln["data_bytes"], "shape": ln["shape"], "proto": proto,
                        "kernel_us": round(us, 2), "GBps": round(alg / us / 1e3, 1),
                        "frac": round(alg / us / 1e3 / PEAK_GBS, 3), "event_us": ln[proto]["us"]})
        text = ["data_bytes shape               proto   kernel_us    GB/s   frac  (event us/launch)"]
        for r in out:
            text.append(f"{r['data_bytes']:>10} {r['shape']:<20} {r['proto']:<6} {r['kernel_us']:>9} {r['GBps']:>8} "
                        f"{r['frac']:>6}  ({r['event_us']})")
    else:
        # gfx950: FETCH_SIZE counts half the bytes of a coalesced streaming read (MI355X_MICROARCH.md,
        # HBM section), WRITE_SIZE is exact; both in KiB
        fetch = {(ln["data_bytes"], ln["shape"], p): statistics.median(v for _, v, _ in seg) * 2048
                 for ln, p, seg in segments(nexr_counters(a.fetch, "FETCH_SIZE"), lines)}
        write = {(ln["data_bytes"], ln["shape"], p): statistics.median(v for _, v, _ in seg) * 1024
                 for ln, p, seg in segments(nexr_counters(a.write, "WRITE_SIZE"), lines)}
        text = ["data_bytes shape               proto   read_B        write_B       alg_B         traffic/alg"]
        for ln in lines:
            for p in ("ll", "ll128", "simple"):
                k = (ln["data_bytes"], ln["shape"], p)
                alg = ln[p]["alg_bytes"]
                out.append({"data_bytes": k[0], "shape": k[1], "proto": p, "read_bytes": int(fetch[k]),
                            "write_bytes": int(write[k]), "alg_bytes": alg,
                            "traffic_over_alg": round((fetch[k] + write[k]) / alg, 4)})
                r = out[-1]
                text.append(f"{k[0]:>10} {k[1]:<20} {p:<6} {r['read_bytes']:>13} {r['write_bytes']:>13} {alg:>13} "
                            f"{r['traffic_over_alg']:>8}")
    body = "\n".join(text)
    print(body)
    if a.out:
        with open(a.out, "w") as f:
            f.write(body + "\n")
    return out


if __name__ == "__main__":
    main()
