#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, a short bench, a rocprof pass.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
stop_if_fatal() {   # $1 = exit status of a GPU step
  case "$1" in
    0|1) return 0 ;;            # ok / test failures: keep going
    *) echo "fatal status $1: stopping"; exit "$1" ;;
  esac
}
python -m metacov_amd.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
s=$?; cat gpurun_out/smoke.log; stop_if_fatal $s
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
s=$?; tail -30 gpurun_out/pytest_gpu.log; stop_if_fatal $s
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
s=$?; tail -5 gpurun_out/bench.log; stop_if_fatal $s
exit 0
