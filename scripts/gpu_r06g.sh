#!/bin/bash
# round 6: the device read pass with kept buffers: experimental tests, the
# experimental bench, and a kernel trace of it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06g}
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_experimental.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/${T}_pytest_exp.log" 2>&1 || { echo "exp tests failed"; tail -30 "$O/${T}_pytest_exp.log"; exit 1; }
tail -1 "$O/${T}_pytest_exp.log"
timeout -k 10 400 python -u scripts/bench_experimental.py --reps 3 > "$O/${T}_experimental.json" 2> "$O/${T}_experimental.err" || { echo "exp bench failed"; tail -20 "$O/${T}_experimental.err"; exit 1; }
cat "$O/${T}_experimental.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${T}_exp" -o run \
    -- python3 "$R/scripts/bench_experimental.py" --reps 3 > "$O/prof_${T}_exp.log" 2>&1 || { echo "trace failed"; tail -5 "$O/prof_${T}_exp.log"; exit 1; }
echo done
