#!/bin/bash
# r03o: speculative long buckets / no end-of-prepare sync: GPU suite, prepare A/B, benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal $1"; exit "$1" ;; esac; }
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/r03o_pytest_gpu.log 2>&1
s=$?; tail -4 $O/r03o_pytest_gpu.log; faulted $O/r03o_pytest_gpu.log; fatal $s
timeout -k 10 300 python scripts/prep_probe.py --config c5 --reps 10 --libs $V/lib_fold.so $V/lib_spec.so > $O/r03o_prep_c5.txt 2>&1
s=$?; grep -v amdgpu.ids $O/r03o_prep_c5.txt; faulted $O/r03o_prep_c5.txt; fatal $s
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/r03o_bench_c5.log 2>&1
s=$?; tail -1 $O/r03o_bench_c5.log | cut -c1-300; faulted $O/r03o_bench_c5.log; fatal $s
timeout -k 10 300 python bench.py > $O/r03o_bench.log 2>&1
s=$?; tail -1 $O/r03o_bench.log | cut -c1-300; faulted $O/r03o_bench.log; fatal $s
exit 0
