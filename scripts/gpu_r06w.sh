#!/bin/bash
# round 6: timing events on the launches (hipExtLaunchKernel) vs hipEventRecord, in process:
# direct C3 / C2 / the N=8 share, fused C5; then the engine GPU tests.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export PYTHONUNBUFFERED=1
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
L="$V/lib_noext.so $V/lib_ext.so"
for m in "direct c2" "direct c3" "fused c5" "direct s8"; do
  set -- $m
  extra="--config $2"; [ $2 = s8 ] && extra="--config c3 --reads 12500000 --contigs 125"
  timeout -k 10 400 python scripts/ab_inproc.py --libs $L --mode $1 $extra --rounds 5 --steps 10 --loop > $O/r06w_ab_$1_$2.txt 2>&1
  s=$?; grep -v amdgpu.ids $O/r06w_ab_$1_$2.txt | tail -4; faulted $O/r06w_ab_$1_$2.txt; [ $s -eq 0 ] || exit $s
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06w_pytest_parity.log 2>&1; s=$?; tail -1 $O/r06w_pytest_parity.log; [ $s -eq 0 ] || exit $s
echo done
