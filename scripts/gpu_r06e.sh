#!/bin/bash
# round 6: full GPU tests, then the cap bench and the cold CLI (fast exit).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06e}
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$O/${T}_pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/${T}_pytest_gpu.log"; exit 1; }
tail -1 "$O/${T}_pytest_gpu.log"
timeout -k 10 500 python -u scripts/cap_bench.py > "$O/${T}_cap_bench.json" 2> "$O/${T}_cap_bench.err" || { echo "cap bench failed"; tail -20 "$O/${T}_cap_bench.err"; exit 1; }
cat "$O/${T}_cap_bench.json"
timeout -k 10 500 python -u scripts/cold_cli.py --runs 3 > "$O/${T}_cold_cli.json" 2> "$O/${T}_cold_cli.err" || { echo "cold cli failed"; tail -20 "$O/${T}_cold_cli.err"; exit 1; }
cat "$O/${T}_cold_cli.json"
