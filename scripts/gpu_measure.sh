#!/bin/bash
# Round-5 measurement session: default bench (C3 + CPU baselines), C2 and C5
# bench lines, then rocprofv3 trace / FETCH_SIZE / WRITE_SIZE passes of each
# (scripts/profile.sh).  Every GPU step has its own limit; the first failure
# ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?set TAG}
O=$R/gpurun_out
mkdir -p "$O"
export PYTHONUNBUFFERED=1
run() { local name=$1; shift; timeout -k 10 ${STEP_LIMIT:-400} "$@" > "$O/${TAG}_$name.log" 2>&1; local s=$?; tail -1 "$O/${TAG}_$name.log" | cut -c1-400; [ $s -ne 0 ] && { echo "$name failed ($s)"; tail -20 "$O/${TAG}_$name.log"; exit $s; }; return 0; }
[ -z "${SKIP_BENCH:-}" ] && run bench python bench.py ${BENCH_ARGS:-}
[ -z "${SKIP_BENCH:-}" ] && run bench_c2 python bench.py --config c2 --no-cpu-baseline
[ -z "${SKIP_BENCH:-}" ] && run bench_c5 python bench.py --config c5 --no-cpu-baseline
for c in ${PROF_CONFIGS:-}; do
  TAG=${TAG}_$c BENCH_ARGS="--config $c" bash "$R/scripts/profile.sh" || exit $?
done
exit 0
