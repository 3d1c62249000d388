#!/bin/bash
# round 6: cold `metacov pileup` wall time with and without the HIP prewarm thread.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
for pw in 1 0 1 0; do
  MC_CLI_PREWARM=$pw timeout -k 10 400 python -u scripts/cold_cli.py --runs 3 > "$O/r06cli2_pw$pw.json" 2> "$O/r06cli2_pw$pw.err" || { echo "cold cli failed"; tail -20 "$O/r06cli2_pw$pw.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('runs') or [{}]; b=min(r, key=lambda x: x.get('wall_s', 9)); print('prewarm', sys.argv[2], 'best wall', round(d['best_wall_s'],3), {k: round(v,3) for k, v in b.items() if k.endswith('_s') and isinstance(v, float)})" "$O/r06cli2_pw$pw.json" $pw
done
echo done
