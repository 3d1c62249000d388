#!/bin/bash
# round 6: cap tests + cap bench (uniform-op walk), experimental bench
# (device vs host read pass), and the benches on the current tree.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06f}
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_depth_cap.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > "$O/${T}_pytest_cap.log" 2>&1 || { echo "cap tests failed"; tail -30 "$O/${T}_pytest_cap.log"; exit 1; }
tail -1 "$O/${T}_pytest_cap.log"
timeout -k 10 400 python -u scripts/cap_bench.py > "$O/${T}_cap_bench.json" 2> "$O/${T}_cap_bench.err" || { echo "cap bench failed"; tail -20 "$O/${T}_cap_bench.err"; exit 1; }
cat "$O/${T}_cap_bench.json"
timeout -k 10 400 python -u scripts/bench_experimental.py --reps 2 > "$O/${T}_experimental.json" 2> "$O/${T}_experimental.err" || { echo "exp bench failed"; tail -20 "$O/${T}_experimental.err"; exit 1; }
cat "$O/${T}_experimental.json"
timeout -k 10 300 python bench.py > "$O/${T}_bench.log" 2>&1 || { echo "bench failed"; tail -5 "$O/${T}_bench.log"; exit 1; }
tail -1 "$O/${T}_bench.log"
for c in c2 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > "$O/${T}_bench_$c.log" 2>&1 || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 200 python bench.py --reads 12500000 --contigs 125 --no-cpu-baseline > "$O/${T}_bench_shard8.log" 2>&1 || exit 1
echo done
