#!/bin/bash
# r03k: histogram A/B (lib_halo -> lib_hist), GPU suite, host probe of the
# stamp build, bench.  Stops on a fault.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal $1"; exit "$1" ;; esac; }
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
TAG=r03k A=$V/lib_halo.so B=$V/lib_hist.so bash scripts/r03_hist_ab.sh
s=$?; [ $s -eq 0 ] || { echo "hist ab status $s"; exit $s; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/r03k_pytest_gpu.log 2>&1
s=$?; tail -4 $O/r03k_pytest_gpu.log; faulted $O/r03k_pytest_gpu.log; fatal $s
timeout -k 10 300 python scripts/host_probe.py --reps 20 --libs $V/lib_hist.so $V/lib_stamp.so > $O/r03k_host.txt 2>&1
s=$?; grep -v amdgpu.ids $O/r03k_host.txt; faulted $O/r03k_host.txt; fatal $s
timeout -k 10 300 python bench.py > $O/r03k_bench.log 2>&1
s=$?; tail -1 $O/r03k_bench.log | cut -c1-400; faulted $O/r03k_bench.log; fatal $s
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/r03k_bench_c5.log 2>&1
s=$?; tail -1 $O/r03k_bench_c5.log | cut -c1-400; faulted $O/r03k_bench_c5.log; fatal $s
exit 0
