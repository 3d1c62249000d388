#!/bin/bash
# round 6: decode / scan GPU tests on the new sources, benches (C3, C2, the
# N=8 share) and a trace + FETCH/WRITE + two SQ passes of the C3 bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06b}
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_scan.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/${T}_pytest.log" 2>&1 || { echo "pytest failed"; tail -20 "$O/${T}_pytest.log"; exit 1; }
tail -1 "$O/${T}_pytest.log"
timeout -k 10 300 python bench.py > "$O/${T}_bench.log" 2>&1 || { echo "bench failed"; tail -5 "$O/${T}_bench.log"; exit 1; }
timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline > "$O/${T}_bench_c2.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --reads 12500000 --contigs 125 --no-cpu-baseline > "$O/${T}_bench_shard8.log" 2>&1 || exit 1
TAG=$T SQ_PASSES="${SQ_PASSES:-A B}" bash scripts/profile.sh
