#!/bin/bash
# round 6: A/B of the fused long-read K2 with deferred tile stores (C5), in process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export PYTHONUNBUFFERED=1
L="metacov_amd/variants/lib_base.so metacov_amd/variants/lib_defer.so"
timeout -k 10 400 python scripts/ab_inproc.py --libs $L --mode fused --config c5 --rounds 5 --steps 8 > $O/r06j_ab_fused_c5.txt 2>&1 || { tail -5 $O/r06j_ab_fused_c5.txt; exit 1; }
grep -v amdgpu.ids $O/r06j_ab_fused_c5.txt
echo done
