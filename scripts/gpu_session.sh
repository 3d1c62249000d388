#!/bin/bash
# One GPU-box session of several steps, each under its own time limit; a
# fault / abort / time limit ends the session (exit codes 0-1 continue).
#   STEPS="tests gz k2ab bench prof" TAG=r04d bash scripts/gpu_session.sh
# tests: pytest -m gpu (PYTEST_SEL narrows it); gz: scripts/gz_ab.py over
# GZ_VARIANTS; k2ab: scripts/gpu_ab_r04.sh with AB_LIBS / AB_RUNS; bench:
# bench.py BENCH_ARGS; prof: scripts/profile.sh (PROF_TAG, BENCH_ARGS).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export PYTHONUNBUFFERED=1
TAG=${TAG:?set TAG}
fatal() { case "$1" in 0|1) return 0 ;; *) echo "step $2: fatal status $1, stopping"; exit "$1" ;; esac; }
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
for step in ${STEPS:-tests}; do
  case $step in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -v --timeout 300 \
          --timeout-method thread -p no:cacheprovider > "$O/${TAG}_pytest_gpu.log" 2>&1
      s=$?; grep -E "passed|failed|error" "$O/${TAG}_pytest_gpu.log" | tail -8; faulted "$O/${TAG}_pytest_gpu.log"; fatal $s tests ;;
    gz)
      timeout -k 10 ${GZ_TIMEOUT:-500} python -u scripts/gz_ab.py --reads ${GZ_READS:-10000000} --reps ${GZ_REPS:-3} --window ${GZ_WINDOW:-0} \
          ${GZ_VARIANTS:?} > "$O/${TAG}_gz_ab.txt" 2>&1
      s=$?; grep -v "^{" "$O/${TAG}_gz_ab.txt" | tail -24; faulted "$O/${TAG}_gz_ab.txt"; fatal $s gz ;;
    k2ab)
      TAG=${TAG}_k2 bash "$R/scripts/gpu_ab_r04.sh"; s=$?; fatal $s k2ab ;;
    bench|bench_c2|bench_c5)
      cfg=""; [ $step = bench_c2 ] && cfg="--config c2"; [ $step = bench_c5 ] && cfg="--config c5 --no-cpu-baseline"
      timeout -k 10 300 python bench.py $cfg ${BENCH_ARGS:-} > "$O/${TAG}_${step}.log" 2>&1
      s=$?; tail -1 "$O/${TAG}_${step}.log" | cut -c1-300; faulted "$O/${TAG}_${step}.log"; fatal $s $step ;;
    smoke)
      timeout -k 10 240 python __graft_entry__.py smoke > "$O/${TAG}_smoke.log" 2>&1
      s=$?; tail -2 "$O/${TAG}_smoke.log"; faulted "$O/${TAG}_smoke.log"; fatal $s smoke ;;
    prof)
      TAG=${PROF_TAG:?} bash "$R/scripts/profile.sh"; s=$?; fatal $s prof ;;
    hostreg) # scripts/micro/hostreg_probe: DMA from a registered page-cache mapping vs pread staging
      head -c $((2048 << 20)) /dev/urandom > /tmp/hostreg.bin && cat /tmp/hostreg.bin > /dev/null
      timeout -k 10 120 "$R/scripts/micro/hostreg_probe" /tmp/hostreg.bin 256 > "$O/${TAG}_hostreg.txt" 2>&1
      s=$?; cat "$O/${TAG}_hostreg.txt"; [ $s -eq 0 ] && timeout -k 10 120 "$R/scripts/micro/hostreg_probe" /tmp/hostreg.bin 64 >> "$O/${TAG}_hostreg.txt" 2>&1
      s=$?; tail -4 "$O/${TAG}_hostreg.txt"; rm -f /tmp/hostreg.bin; faulted "$O/${TAG}_hostreg.txt"; fatal $s hostreg ;;
    e2e)     # scripts/e2e.py: CLI end to end, host and GPU decode of one 30 M-record BAM
      mkdir -p /tmp/e2e
      timeout -k 10 600 python scripts/e2e.py --reads ${E2E_READS:-30000000} --contigs 1000 --length 1000000 \
          --dir /tmp/e2e ${E2E_ARGS:-} > "$O/${TAG}_e2e.json" 2> "$O/${TAG}_e2e.err"
      s=$?; tail -3 "$O/${TAG}_e2e.err"; python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['gpu_decode_s'],d['gpu_end_to_end_s'],d['gpu_decode_timings'])" "$O/${TAG}_e2e.json"
      faulted "$O/${TAG}_e2e.err"; fatal $s e2e ;;
    gzpmc)   # kernel trace + SQ counter passes over one GPU decode (variant GZ_PMC_VARIANT)
      G="$R/scripts/gz_ab.py --reads ${GZ_PMC_READS:-3000000} --reps 1 ${GZ_PMC_VARIANT:-gzopq}"
      ( cd /tmp && export TMPDIR=/tmp
        timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof_${TAG}_gz_trace" -o run \
            -- python3 $G > "$O/prof_${TAG}_gz_trace.log" 2>&1 || exit 1
        for p in A B; do
          case $p in
            A) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY" ;;
            B) C="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM" ;;
          esac
          timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$O/prof_${TAG}_gz_sq$p" -o run \
              -- python3 $G > "$O/prof_${TAG}_gz_sq$p.log" 2>&1 || exit 1
        done )
      s=$?; python3 "$R/scripts/sq_summary.py" ${TAG}_gz gz_inflate 2>&1 | tail -20; fatal $s gzpmc ;;
  esac
done
exit 0
