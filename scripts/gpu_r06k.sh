#!/bin/bash
# round 6: A/B of K2 builds: base, deferred stores in the fused long K2, and
# 2048-position tiles (with deferral); fused C5 and direct C3, in process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export PYTHONUNBUFFERED=1
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
L="$V/lib_base.so $V/lib_defer.so $V/lib_t2k.so"
for m in "fused c5" "direct c3" "fused c3"; do
  set -- $m
  timeout -k 10 400 python scripts/ab_inproc.py --libs $L --mode $1 --config $2 --rounds 4 --steps 8 > $O/r06k_ab_$1_$2.txt 2>&1
  s=$?; grep -v amdgpu.ids $O/r06k_ab_$1_$2.txt | tail -6; faulted $O/r06k_ab_$1_$2.txt; [ $s -eq 0 ] || exit $s
done
echo done
