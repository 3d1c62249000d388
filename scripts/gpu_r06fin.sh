#!/bin/bash
# round 6, final tree: the GPU suite, smoke, the benches (C3, C2, C5, one N=8
# share, scan) and the PMC passes (scripts/gpu_r06fin_pmc.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=r06fin
cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/${T}_pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/${T}_pytest_gpu.log"; exit 1; }
tail -1 "$O/${T}_pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/${T}_smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/${T}_smoke.log"; exit 1; }
tail -1 "$O/${T}_smoke.log"
timeout -k 10 300 python bench.py > "$O/${T}_bench.log" 2>&1 || { echo "bench failed"; tail -5 "$O/${T}_bench.log"; exit 1; }
for c in c2 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > "$O/${T}_bench_$c.log" 2>&1 || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 200 python bench.py --reads 12500000 --contigs 125 --no-cpu-baseline > "$O/${T}_bench_shard8.log" 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_scan.py > "$O/${T}_scan_bench.log" 2>&1 || { echo "scan bench failed"; exit 1; }
for f in bench bench_c2 bench_c5 bench_shard8 scan_bench; do
  python - "$O/${T}_$f.log" $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 4), "%.4g" % d["value"], d.get("kernels_ms"), (d.get("roofline") or {}).get("traffic"))
PY
done
bash scripts/gpu_r06fin_pmc.sh || exit 1
echo done
