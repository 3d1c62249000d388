#!/bin/bash
# A/B of K2 builds (LIBS="a.so b.so ..."): direct (C3), fused on the packed words (C3), fused C5;
# then the GPU tests of the histogram path.  Stops on a fault.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${TAG:?set TAG}
LIBS=${LIBS:?libs to compare}
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal $1"; exit "$1" ;; esac; }
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "fused or stats or direct" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/${TAG}_tests.log 2>&1
s=$?; tail -3 $O/${TAG}_tests.log; faulted $O/${TAG}_tests.log; fatal $s
for m in "direct c3" "fused c3" "fused c5"; do
  set -- $m
  timeout -k 10 400 python scripts/ab_inproc.py --libs $LIBS --mode $1 --config $2 --rounds 4 --steps 8 > $O/${TAG}_ab_$1_$2.txt 2>&1
  s=$?; grep -v amdgpu.ids $O/${TAG}_ab_$1_$2.txt; faulted $O/${TAG}_ab_$1_$2.txt; fatal $s
done
exit 0
