#!/bin/bash
# round-3 combined session: direct-path A/B (C3), long-read histogram A/B (C5), GPU tests
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${TAG:-r03i}
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal $1"; exit "$1" ;; esac; }
# a GPU fault reported through Python (exit status 1) also ends the session
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
# the kernels that faulted in r03e first, alone
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k 'direct or library_then_torch or device_recompute' -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/${TAG}_risky.log 2>&1
s=$?; grep -E "PASS|FAIL|passed|failed|Error" $O/${TAG}_risky.log | tail -12; faulted $O/${TAG}_risky.log; fatal $s
timeout -k 10 400 python scripts/ab_inproc.py --libs $V/lib_ord64.so $V/lib_halo.so --mode direct --rounds 4 --steps 10 > $O/${TAG}_ab_c3.txt 2>&1
s=$?; grep -v amdgpu.ids $O/${TAG}_ab_c3.txt; faulted $O/${TAG}_ab_c3.txt; fatal $s
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${TAG}_pytest_gpu.log 2>&1
s=$?; grep -E "passed|failed|FAILED" $O/${TAG}_pytest_gpu.log | tail -5; faulted $O/${TAG}_pytest_gpu.log; fatal $s
timeout -k 10 300 python bench.py > $O/${TAG}_bench.log 2>&1
s=$?; tail -1 $O/${TAG}_bench.log | cut -c1-600; faulted $O/${TAG}_bench.log; fatal $s
exit 0
