#!/bin/bash
# One GPU-box session with the prebuilt in-tree .so: smoke, GPU parity tests,
# bench, optionally rocprofv3 kernel-trace stats of the bench.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r03}
O=$R/gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
stop_if_fatal() {
  case "$1" in
    0|1) return 0 ;;
    *) echo "fatal status $1: stopping"; exit "$1" ;;
  esac
}
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 240 python __graft_entry__.py smoke > $O/${TAG}_smoke.log 2>&1
s=$?; cat $O/${TAG}_smoke.log; faulted $O/${TAG}_smoke.log; stop_if_fatal $s
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu ${PYTEST_ARGS:--x} -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${TAG}_pytest_gpu.log 2>&1
s=$?; grep -E "passed|failed|error" $O/${TAG}_pytest_gpu.log | tail -15; faulted $O/${TAG}_pytest_gpu.log; stop_if_fatal $s
fi
if [ -z "${SKIP_BENCH:-}" ]; then
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/${TAG}_bench.log 2>&1
s=$?; tail -2 $O/${TAG}_bench.log; faulted $O/${TAG}_bench.log; stop_if_fatal $s
fi
if [ -n "${PROF:-}" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/${TAG}_prof.log 2>&1
s=$?; tail -2 $O/${TAG}_prof.log; faulted $O/${TAG}_prof.log; stop_if_fatal $s
cd $R
fi
exit 0
