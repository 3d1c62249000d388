#!/bin/bash
# SQ-counter pass over the fused and unfused bench (one rocprofv3 pass each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1 || true
for mode in fused unfused; do
  extra=""; [ $mode = unfused ] && extra="--unfused"
  timeout -k 10 300 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY} \
      --output-format csv -d "$R/gpurun_out/sq_$mode" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $extra \
      > "$R/gpurun_out/sq_$mode.log" 2>&1 || { echo "pass $mode failed"; tail -5 "$R/gpurun_out/sq_$mode.log"; exit 1; }
done
