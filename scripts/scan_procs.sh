#!/bin/bash
# Per-processor timing of the scan kernel (20M reads each).
set -u
mkdir -p gpurun_out
for p in ${PROCS:-base kmer mirror isize base,kmer,mirror,isize}; do
  timeout -k 10 120 python scripts/bench_scan.py --reads 20000000 --steps 3 --no-cpu-baseline --check ${CHECK:-0} --procs $p > gpurun_out/procs_$p.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/procs_$p.log').read().strip().splitlines()[-1]); print('$p', round(d['kernels_ms']['scan_kernel'],2),'ms')"
done
