#!/bin/bash
# rocprofv3 passes over the bench, for scripts/pmc_summary.py <TAG>:
#   trace  --kernel-trace --stats (per-kernel average durations)
#   fetch  --pmc FETCH_SIZE        write  --pmc WRITE_SIZE
# (separate passes: FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2).
# Extra bench flags in BENCH_ARGS (e.g. --unfused, --config c5).  Each pass
# has its own time limit; the first failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?set TAG}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps ${PROF_STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${TAG}_trace" -o run \
    -- python3 $B > "$O/prof_${TAG}_trace.log" 2>&1 || { echo "trace pass failed"; tail -5 "$O/prof_${TAG}_trace.log"; exit 1; }
tail -1 "$O/prof_${TAG}_trace.log"
for c in FETCH_SIZE WRITE_SIZE; do
  d=fetch; [ $c = WRITE_SIZE ] && d=write
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$O/prof_${TAG}_$d" -o run \
      -- python3 $B > "$O/prof_${TAG}_$d.log" 2>&1 || { echo "$c pass failed"; tail -5 "$O/prof_${TAG}_$d.log"; exit 1; }
done
for p in ${SQ_PASSES:-}; do   # SQ_PASSES="A B": SQ counter sets below
  case $p in
    A) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY" ;;
    B) C="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM" ;;
  esac
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$O/prof_${TAG}_sq$p" -o run \
      -- python3 $B > "$O/prof_${TAG}_sq$p.log" 2>&1 || { echo "SQ pass $p failed"; tail -5 "$O/prof_${TAG}_sq$p.log"; exit 1; }
done
exit 0
