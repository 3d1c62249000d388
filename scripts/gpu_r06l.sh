#!/bin/bash
# round 6: A/B of the fused direct K2 with deferred tile stores (C3, C2), in process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export PYTHONUNBUFFERED=1
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
L="$V/lib_base.so $V/lib_ddir.so $V/lib_ns.so $V/lib_nsd.so"
for m in "direct c3" "direct c2"; do
  set -- $m
  timeout -k 10 400 python scripts/ab_inproc.py --libs $L --mode $1 --config $2 --rounds 6 --steps 8 > $O/r06l_ab_$1_$2.txt 2>&1
  s=$?; grep -v amdgpu.ids $O/r06l_ab_$1_$2.txt | tail -4; faulted $O/r06l_ab_$1_$2.txt; [ $s -eq 0 ] || exit $s
done
echo done
