#!/bin/bash
# round 6: device cap (tests + scripts/cap_bench.py) and the cold CLI record.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06c}
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_depth_cap.py tests/test_npstd.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "cap or capped" > "$O/${T}_pytest_cap.log" 2>&1 || { echo "cap tests failed"; tail -30 "$O/${T}_pytest_cap.log"; exit 1; }
tail -1 "$O/${T}_pytest_cap.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "pysam or classic_defaults or capped" > "$O/${T}_pytest_parity.log" 2>&1 || { echo "parity tests failed"; tail -30 "$O/${T}_pytest_parity.log"; exit 1; }
tail -1 "$O/${T}_pytest_parity.log"
timeout -k 10 500 python -u scripts/cap_bench.py > "$O/${T}_cap_bench.json" 2> "$O/${T}_cap_bench.err" || { echo "cap bench failed"; tail -20 "$O/${T}_cap_bench.err"; exit 1; }
cat "$O/${T}_cap_bench.json"
timeout -k 10 500 python -u scripts/cold_cli.py --runs 3 > "$O/${T}_cold_cli.json" 2> "$O/${T}_cold_cli.err" || { echo "cold cli failed"; tail -20 "$O/${T}_cold_cli.err"; exit 1; }
cat "$O/${T}_cold_cli.json"
# scan: SQ counters of the final scan kernels (all four tables)
TAG=${T}_scan SCAN_PROCS=${SCAN_PROCS:-base,kmer,mirror,isize} bash scripts/gpu_scan_sq.sh || exit 1
python3 scripts/sq_scan_summary.py ${T}_scan libmetacov_amd > "$O/${T}_sq_scan.json" || exit 1
timeout -k 10 300 python scripts/bench_scan.py > "$O/${T}_scan_bench.log" 2>&1 || { echo "scan bench failed"; tail -5 "$O/${T}_scan_bench.log"; exit 1; }
tail -1 "$O/${T}_scan_bench.log"
