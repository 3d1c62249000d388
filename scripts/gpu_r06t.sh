#!/bin/bash
# round 6: the GPU suite, smoke and the bench / scan bench on the current tree.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06t}
cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/${T}_pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/${T}_pytest_gpu.log"; exit 1; }
tail -1 "$O/${T}_pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/${T}_smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/${T}_smoke.log"; exit 1; }
tail -1 "$O/${T}_smoke.log"
timeout -k 10 300 python bench.py > "$O/${T}_bench.log" 2>&1 || { echo "bench failed"; tail -5 "$O/${T}_bench.log"; exit 1; }
tail -1 "$O/${T}_bench.log" | cut -c1-400
timeout -k 10 300 python scripts/bench_scan.py > "$O/${T}_scan_bench.log" 2>&1 || { echo "scan bench failed"; tail -5 "$O/${T}_scan_bench.log"; exit 1; }
tail -1 "$O/${T}_scan_bench.log" | cut -c1-300
echo done
