#!/bin/bash
# r03n: folded long-read counting: tests, prepare A/B (C5, C3), C5 bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal $1"; exit "$1" ;; esac; }
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "long or ont or folded or c5" tests/test_gpu_fullsize.py -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf > $O/r03n_tests.log 2>&1
s=$?; tail -4 $O/r03n_tests.log; faulted $O/r03n_tests.log; fatal $s
timeout -k 10 300 python scripts/prep_probe.py --config c5 --reps 10 --libs $V/lib_stamp.so $V/lib_fold.so > $O/r03n_prep_c5.txt 2>&1
s=$?; grep -v amdgpu.ids $O/r03n_prep_c5.txt; faulted $O/r03n_prep_c5.txt; fatal $s
timeout -k 10 300 python scripts/prep_probe.py --config c3 --reps 10 --libs $V/lib_stamp.so $V/lib_fold.so > $O/r03n_prep_c3.txt 2>&1
s=$?; grep -v amdgpu.ids $O/r03n_prep_c3.txt; faulted $O/r03n_prep_c3.txt; fatal $s
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/r03n_bench_c5.log 2>&1
s=$?; tail -1 $O/r03n_bench_c5.log | cut -c1-300; faulted $O/r03n_bench_c5.log; fatal $s
exit 0
