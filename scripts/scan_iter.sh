#!/bin/bash
# One scan iteration on the GPU: parity tests, then per-processor timings.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_scan.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/scan_iter_tests.log 2>&1
s=$?; tail -3 gpurun_out/scan_iter_tests.log; [ $s -eq 0 ] || exit $s
bash scripts/scan_procs.sh
