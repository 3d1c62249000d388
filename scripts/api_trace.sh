#!/bin/bash
# HIP API + kernel trace of a short bench run (no counters), for
# scripts/api_gaps.py: where the host time between two steps goes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?set TAG}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$O/prof_${TAG}_api" -o run \
    -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --prepare-steps 0 ${BENCH_ARGS:-} \
    > "$O/prof_${TAG}_api.log" 2>&1 || { echo "api trace failed"; tail -5 "$O/prof_${TAG}_api.log"; exit 1; }
tail -1 "$O/prof_${TAG}_api.log" | cut -c1-300
