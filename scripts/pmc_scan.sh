#!/bin/bash
# SQ-counter passes over the scan bench (one rocprofv3 pass per counter set).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/pmc_scan$i" -o run -- \
      python3 "$R/scripts/bench_scan.py" --reads 20000000 --steps 1 --warmup 0 --check 0 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$R/gpurun_out/pmc_scan$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc_scan$i.log"; exit 1; }
  python3 - "$R/gpurun_out/pmc_scan$i" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(float)
for r in rows:
    if "scan_kernel" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print("%-24s %.4g" % (k, v))
PY
done
