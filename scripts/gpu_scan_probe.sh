#!/bin/bash
# scan_kernel breakdown: bench_scan per processor set, then SQ counter passes
# of the full set (each GPU step under its own limit; the first failure ends
# the script).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?set TAG}
O=$R/gpurun_out
mkdir -p "$O"
export PYTHONUNBUFFERED=1
N=${SCAN_READS:-20000000}
for p in ${SCAN_PROCS:-base,kmer,mirror,isize base kmer mirror isize}; do
  timeout -k 10 300 python scripts/bench_scan.py --reads $N --steps 5 --no-cpu-baseline --check ${SCAN_CHECK:-0} --procs $p \
      > "$O/${TAG}_scan_$p.log" 2>&1 || { echo "bench_scan $p failed"; tail -5 "$O/${TAG}_scan_$p.log"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['kernels_ms'])" "$O/${TAG}_scan_$p.log" $p
done
if [ -n "${SCAN_SQ:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  B="$R/scripts/bench_scan.py --reads $N --steps 2 --warmup 1 --no-cpu-baseline --check 0"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
      --output-format csv -d "$O/prof_${TAG}_scan_sqA" -o run -- python3 $B > "$O/prof_${TAG}_scan_sqA.log" 2>&1 || { echo "sqA failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM \
      --output-format csv -d "$O/prof_${TAG}_scan_sqB" -o run -- python3 $B > "$O/prof_${TAG}_scan_sqB.log" 2>&1 || { echo "sqB failed"; exit 1; }
fi
exit 0
