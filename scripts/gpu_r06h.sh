#!/bin/bash
# round 6: tile-grouped stores in the long-read fill (MC_FILL_SORTED): the
# GPU suite, C5 / C3 benches and a C5 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06h}
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/${T}_pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/${T}_pytest_gpu.log"; exit 1; }
tail -1 "$O/${T}_pytest_gpu.log"
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > "$O/${T}_bench_c5.log" 2>&1 || { echo "bench c5 failed"; tail -5 "$O/${T}_bench_c5.log"; exit 1; }
tail -1 "$O/${T}_bench_c5.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/${T}_bench.log" 2>&1 || { echo "bench failed"; tail -5 "$O/${T}_bench.log"; exit 1; }
tail -1 "$O/${T}_bench.log"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_${T}_c5" -o run -- python3 bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 3 > "$O/${T}_prof_c5.log" 2>&1 || { echo "prof failed"; tail -5 "$O/${T}_prof_c5.log"; exit 1; }
echo done
