#!/bin/bash
# Round-4 A/B session: in-process A/B of K2 build variants (metacov_amd/variants)
# on C3 (direct + fused), C5 (fused) and C2 (direct), then optional rocprofv3
# passes of one config.  Each GPU step has its own time limit; the first
# failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04ab}
LIBS="metacov_amd/libmetacov_amd.so ${AB_LIBS:-}"
for spec in ${AB_RUNS:-c3:direct c3:fused c5:fused c2:direct}; do
  cfg=${spec%%:*}; mode=${spec##*:}
  timeout -k 10 ${AB_TIMEOUT:-240} python scripts/ab_inproc.py --libs $LIBS --config $cfg --mode $mode \
      --rounds ${AB_ROUNDS:-4} --steps ${AB_STEPS:-10} ${AB_EXTRA:-} > "$O/${TAG}_${cfg}_${mode}.txt" 2>&1
  s=$?; tail -${AB_TAIL:-6} "$O/${TAG}_${cfg}_${mode}.txt"; [ $s -ne 0 ] && { echo "A/B $spec failed ($s)"; exit $s; }
done
if [ -n "${PROF_TAG:-}" ]; then
  TAG=$PROF_TAG bash "$R/scripts/profile.sh" || exit $?
fi
exit 0
