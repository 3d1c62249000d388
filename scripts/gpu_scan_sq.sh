#!/bin/bash
# SQ counter passes of bench_scan for each library in SCAN_LIBS and processor
# set SCAN_PROCS (one rocprofv3 --pmc run per counter set; each under its own
# limit; the first failure ends the script).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?set TAG}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for lib in ${SCAN_LIBS:-metacov_amd/libmetacov_amd.so}; do
  n=$(basename $lib .so)
  export METACOV_AMD_LIB=$R/$lib
  B="$R/scripts/bench_scan.py --reads ${SCAN_READS:-100000000} --steps 1 --warmup 0 --no-cpu-baseline --check 0 --procs ${SCAN_PROCS:-mirror}"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      --output-format csv -d "$O/prof_${TAG}_${n}" -o run -- python3 $B > "$O/prof_${TAG}_${n}.log" 2>&1 || { echo "$n failed"; tail -5 "$O/prof_${TAG}_${n}.log"; exit 1; }
  python3 - "$O/prof_${TAG}_${n}/run_counter_collection.csv" $n <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'scan_kernel' in r['Kernel_Name']:
        agg[r['Counter_Name']] += float(r['Counter_Value'])
print(sys.argv[2], {k: '%.3g' % v for k, v in sorted(agg.items())})
PY
done
