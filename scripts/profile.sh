#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then one
# PMC pass per TCC counter (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r01}
ARGS=${PROF_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
python3 -m metacov_amd.build >/dev/null 2>&1 || (cd "$R" && python3 -m metacov_amd.build)
run() {   # $1 = name, rest = rocprofv3 options
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$R/gpurun_out/prof_${TAG}_${name}" -o run \
      -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof_${TAG}_${name}.log" 2>&1
  local s=$?
  tail -3 "$R/gpurun_out/prof_${TAG}_${name}.log"
  if [ $s -ne 0 ]; then echo "step $name failed with $s"; exit $s; fi
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
exit 0
