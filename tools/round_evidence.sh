#!/bin/bash
# Reproduce a round's headline evidence on one MI355X in one go (run from the repository root, after
# build(); every GPU step under its own time limit, chained so the first failure ends the script):
#   0. a 120 s random parity sweep against the C oracle (tools/fuzz_long.py)
#                                              -> gpurun_out/evidence_<tag>/fuzz.json
#   1. the GPU test suite                      -> gpurun_out/evidence_<tag>/gpu_tests.txt
#   2. smoke()                                 -> .../smoke.txt
#   3. the default bench line                  -> .../bench.json
#   4. rocprofv3 kernel trace of the same bench command, summarised against the line it printed
#                                              -> .../c2_kernel_{trace,stats}.csv, summary.txt
#   5. HBM traffic (FETCH_SIZE / WRITE_SIZE, one rocprofv3 pass per counter) of all nine configurations
#                                              -> profiles/pmc_<config>.json via tools/run_pmc.sh
#   bash tools/round_evidence.sh <tag>
set -o pipefail
tag=${1:?usage: tools/round_evidence.sh <tag>}
out=gpurun_out/evidence_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python tools/fuzz_long.py --seconds 120 --max-mib 200 --budget-mib 2000 > "$out/fuzz.json" 2> "$out/fuzz.err" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$out/gpu_tests.txt" 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o c2 -- \
  python3 bench.py > "$out/bench_under_rocprof.json" 2> "$out/bench_under_rocprof.err" || exit 1
cp "$out/prof/c2_kernel_trace.csv" "$out/prof/c2_kernel_stats.csv" "$out/" || exit 1
python3 tools/prof_summary.py --trace "$out/c2_kernel_trace.csv" --bench "$out/bench_under_rocprof.json" \
  --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py" --out "$out/summary.txt" || exit 1
bash tools/run_pmc.sh "$tag" c2 c3_f16 c3_bf16 c4_i32_min c4_i32_max c4_i32_prod c4_i8_min c4_i8_max c4_i8_prod \
  > "$out/pmc.log" 2>&1 || exit 1
echo "evidence $tag complete" | tee "$out/done.txt"
