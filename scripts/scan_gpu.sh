#!/bin/bash
# scan GPU session: parity tests, the scan bench, a rocprofv3 kernel trace.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-scan}
timeout -k 10 300 python -u -m pytest tests/test_scan.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu.log 2>&1
s=$?; tail -5 gpurun_out/${TAG}_gpu.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python scripts/bench_scan.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
s=$?; tail -3 gpurun_out/${TAG}_bench.log; [ $s -eq 0 ] || exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_scan.py --steps 3 --no-cpu-baseline --check 0 ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1
s=$?; tail -2 $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log; exit $s
