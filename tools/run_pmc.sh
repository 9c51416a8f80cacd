#!/bin/bash
# HBM traffic of the reduce-copy kernel for bench configurations, one rocprofv3 PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), each pass under its own hard limit.
#   bash tools/run_pmc.sh <tag> <config> [<config> ...]
# -> gpurun_out/pmc_<tag>/<config>_{fetch,write}_counter_collection.csv and profiles/pmc_<config>.json
set -o pipefail
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
for cfg in "$@"; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    name=${cfg}_$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$out" -o "$name" -- \
      python3 bench.py --config "$cfg" --steps 5 --warmup 2 --no-cpu --no-h2d --no-extra > "$out/$name.log" 2>&1 || exit 1
  done
  cp "$out/${cfg}_fetch_counter_collection.csv" "profiles/${tag}_${cfg}_pmc_fetch.csv" || exit 1
  cp "$out/${cfg}_write_counter_collection.csv" "profiles/${tag}_${cfg}_pmc_write.csv" || exit 1
  python3 tools/pmc_traffic.py --config "$cfg" --fetch "profiles/${tag}_${cfg}_pmc_fetch.csv" \
    --write "profiles/${tag}_${cfg}_pmc_write.csv" --out "profiles/pmc_$cfg.json" || exit 1
done
mkdir -p gpurun_out/profiles_new && cp profiles/pmc_*.json profiles/${tag}_*_pmc_*.csv gpurun_out/profiles_new/
