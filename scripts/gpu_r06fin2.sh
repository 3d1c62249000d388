#!/bin/bash
# round 6, final tree: cap bench, cold CLI wall time, experimental bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=r06fin
cd "$R"
timeout -k 10 500 python -u scripts/cap_bench.py > "$O/${T}_cap_bench.json" 2> "$O/${T}_cap_bench.err" || { echo "cap bench failed"; tail -20 "$O/${T}_cap_bench.err"; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: v for k, v in d.items() if not isinstance(v, (list, dict))})" "$O/${T}_cap_bench.json"
timeout -k 10 500 python -u scripts/cold_cli.py --runs 3 > "$O/${T}_cold_cli.json" 2> "$O/${T}_cold_cli.err" || { echo "cold cli failed"; tail -20 "$O/${T}_cold_cli.err"; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('cold cli best wall', d['best_wall_s'])" "$O/${T}_cold_cli.json"
timeout -k 10 400 python -u scripts/bench_experimental.py --reps 3 > "$O/${T}_experimental.json" 2> "$O/${T}_experimental.err" || { echo "exp bench failed"; tail -20 "$O/${T}_experimental.err"; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('experimental best', d['best'])" "$O/${T}_experimental.json"
echo done
