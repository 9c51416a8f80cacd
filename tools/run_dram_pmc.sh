#!/bin/bash
# DRAM-side request, occupancy and stall counters of the stream-mix probe (tools/streams.hip) and of
# the C3 bf16 kernel, one rocprofv3 pass per counter group (<= 4 TCC counters per pass on gfx950).
#   bash tools/run_dram_pmc.sh  -> gpurun_out/dram_pmc/<pass>_{streams,c3}_counter_collection.csv
set -o pipefail
out=gpurun_out/dram_pmc
mkdir -p "$out"
export TMPDIR=/tmp
P1="TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ TCC_EA0_WRREQ_LEVEL GRBM_GUI_ACTIVE"
P2="TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL TCC_EA0_RDREQ_DRAM GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $pass --output-format csv -d "$out" -o p${i}_streams -- ./tools/streams 2 \
    > "$out/p${i}_streams.log" 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$out" -o p${i}_c3 -- \
    python3 bench.py --config c3_bf16 --steps 5 --warmup 2 --no-cpu --no-h2d > "$out/p${i}_c3.log" 2>&1 || exit 1
done
