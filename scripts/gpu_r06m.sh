#!/bin/bash
# round 6: the GPU suite and the benches (C3, C2, C5, one N=8 share) on the
# current tree (no VGPR spills in the direct K2, deferred stores in the long K2,
# k-mer codes from 8-base windows) and the scan bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${T:-r06m}
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/${T}_pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/${T}_pytest_gpu.log"; exit 1; }
tail -1 "$O/${T}_pytest_gpu.log"
timeout -k 10 300 python bench.py > "$O/${T}_bench.log" 2>&1 || { echo "bench failed"; tail -5 "$O/${T}_bench.log"; exit 1; }
tail -1 "$O/${T}_bench.log"
for c in c2 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > "$O/${T}_bench_$c.log" 2>&1 || { echo "bench $c failed"; exit 1; }
  tail -1 "$O/${T}_bench_$c.log"
done
timeout -k 10 200 python bench.py --reads 12500000 --contigs 125 --no-cpu-baseline > "$O/${T}_bench_shard8.log" 2>&1 || exit 1
tail -1 "$O/${T}_bench_shard8.log"
timeout -k 10 300 python scripts/bench_scan.py > "$O/${T}_scan_bench.log" 2>&1 || { echo "scan bench failed"; tail -5 "$O/${T}_scan_bench.log"; exit 1; }
tail -1 "$O/${T}_scan_bench.log"
echo done
