#!/bin/bash
# round 6: C2 / C3 direct K2 sensitivity to the next-batch prefetch (in process).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export PYTHONUNBUFFERED=1
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
L=${LIBS:-"$V/lib_base.so $V/lib_pf0.so"}
T=${T:-r06r}
for m in ${CASES:-direct:c2 direct:c3}; do
  set -- ${m/:/ }
  timeout -k 10 400 python scripts/ab_inproc.py --libs $L --mode $1 --config $2 --rounds 5 --steps 10 > $O/${T}_ab_$1_$2.txt 2>&1
  s=$?; grep -v amdgpu.ids $O/${T}_ab_$1_$2.txt | tail -4; faulted $O/${T}_ab_$1_$2.txt; [ $s -eq 0 ] || exit $s
done
echo done
