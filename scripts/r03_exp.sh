#!/bin/bash
# round-3 experiment session: in-process A/B of K2 variants + a kernel trace of the bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${TAG:-r03b}
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal $1"; exit "$1" ;; esac; }
# a GPU fault reported through Python (exit status 1) also ends the session
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
if [ -n "${AB_LIBS:-}" ]; then
timeout -k 10 400 python scripts/ab_inproc.py --libs $AB_LIBS --mode ${AB_MODE:-all} --rounds ${AB_ROUNDS:-4} --steps 10 ${AB_ARGS:-} > $O/${TAG}_ab.txt 2>&1
s=$?; cat $O/${TAG}_ab.txt | grep -v amdgpu.ids; faulted $O/${TAG}_ab.txt; fatal $s
fi
if [ -n "${TRACE:-}" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/${TAG}_trace.log 2>&1
s=$?; tail -1 $O/${TAG}_trace.log | cut -c1-300; faulted $O/${TAG}_trace.log; fatal $s
cd $R
fi
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${TAG}_tests.log 2>&1
s=$?; grep -E "passed|failed" $O/${TAG}_tests.log | tail -3; faulted $O/${TAG}_tests.log; fatal $s
fi
exit 0
