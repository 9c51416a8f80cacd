#!/bin/bash
# HBM traffic of the LL / LL128 / SIMPLE step kernels at 64 MiB per step (tools/ll_rate.py), one
# rocprofv3 PMC pass per counter, each pass under its own hard limit:
#   bash tools/ll_pmc.sh <tag>   -> profiles/<tag>_ll_pmc.txt
set -o pipefail
tag=${1:?usage: tools/ll_pmc.sh <tag>}
out=gpurun_out/ll_pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  name=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out" -o "$name" -- \
    python3 tools/ll_rate.py --sizes 67108864 --reps 3 > "$out/$name.jsonl" 2> "$out/$name.err" || exit 1
done
python3 tools/ll_prof_summary.py --fetch "$out/fetch_counter_collection.csv" --write "$out/write_counter_collection.csv" \
  --rate "$out/fetch.jsonl" --out "$out/${tag}_ll_pmc.txt" || exit 1
