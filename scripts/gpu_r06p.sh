#!/bin/bash
# round 6: scan per processor (100 M reads, one box), after the k-mer window codes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
for p in base kmer mirror isize; do
  timeout -k 10 200 python scripts/bench_scan.py --procs $p --no-cpu-baseline --check 0 > "$O/r06p_scan_$p.log" 2>&1 || { echo "$p failed"; tail -5 "$O/r06p_scan_$p.log"; exit 1; }
  python - "$O/r06p_scan_$p.log" $p <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 3), d["kernels_ms"])
PY
done
echo done
