#!/bin/bash
# A/B of library builds on the bench (same process order, alternating).
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for lib in metacov_amd/libmetacov_amd.so ${AB_LIBS:-}; do
    MC_BENCH_NOCHECK=1 METACOV_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/ab.json 2>/dev/null
    s=$?; [ $s -ne 0 ] && { echo "fail $s $lib"; exit $s; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$lib', d['kernels_ms'], round(d['ms_per_step'],3))"
  done
done
