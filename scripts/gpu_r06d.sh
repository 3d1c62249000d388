#!/bin/bash
# round 6: device cap + device experimental read pass (tests), then the cap
# bench, the cold CLI record and the scan SQ passes (scripts/gpu_r06c.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06d}
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_experimental.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > "$O/${T}_pytest_exp.log" 2>&1 || { echo "exp tests failed"; tail -40 "$O/${T}_pytest_exp.log"; exit 1; }
tail -1 "$O/${T}_pytest_exp.log"
T=$T bash scripts/gpu_r06c.sh
