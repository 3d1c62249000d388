#!/bin/bash
# round 6, last check of the committed tree: the GPU suite and smoke.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/r06final_pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/r06final_pytest_gpu.log"; exit 1; }
tail -1 "$O/r06final_pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/r06final_smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/r06final_smoke.log"; exit 1; }
tail -1 "$O/r06final_smoke.log"
timeout -k 10 300 python bench.py > "$O/r06final_bench.log" 2>&1 || { echo "bench failed"; exit 1; }
tail -1 "$O/r06final_bench.log" | cut -c1-260
echo done
