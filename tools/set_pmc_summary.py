#!/usr/bin/env python3
"""Per-set counter summary of a `rocprofv3 --pmc ... -- python3 tools/tlb_probe.py` pass: the
probe's phase-1 timing (its JSON lines in the step log) next to the mean of every counter over each
set's dispatches (phase 1 round-robin + phase 2 in set order), sets sorted by time.

    python tools/set_pmc_summary.py <step log> <counter_collection.csv> [--sets N --rounds R --reps P]"""
import argparse
import collections
import csv
import json


def summarize(log_path, csv_path, sets, rounds, reps):
    timing = {}
    for ln in open(log_path):
        if ln.startswith("{") and '"set"' in ln:
            d = json.loads(ln)
            timing[d["set"]] = d["median_us"]
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(csv_path)):
        if "reduce_copy" in r["Kernel_Name"]:
            by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)
    per_set = collections.defaultdict(lambda: collections.defaultdict(list))
    for j, d in enumerate(ids):
        s = j % sets if j < sets * rounds else (j - sets * rounds) // reps
        for k, v in by[d].items():
            per_set[s][k].append(v)
    out = []
    for s in sorted(timing, key=timing.get):
        row = {"set": s, "median_us_under_pmc": timing[s]}
        row.update({k: round(sum(v) / len(v), 1) for k, v in sorted(per_set[s].items())})
        out.append(row)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("csv")
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for row in summarize(a.log, a.csv, a.sets, a.rounds, a.reps):
        print(json.dumps(row))
