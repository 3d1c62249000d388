#!/bin/bash
# Host cost of the bench's per-step RCCL exchange: one torchrun rank on the
# N=8 share, with (MC_BENCH_FORCE_EXCHANGE=1) and without the all-gather, one
# all-gather per step (--exchange-every 1) or per 8 steps.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "0 8" "1 1" "1 8" "0 8" "1 1" "1 8"; do
  set -- $cfg; ex=$1; G=$2
  MC_BENCH_FORCE_EXCHANGE=$ex timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --backend nccl --config c3 \
      --reads 12500000 --contigs 125 --steps 40 --warmup 5 --prepare-steps 0 --no-cpu-baseline --exchange-every $G > "$O/exch_$ex.log" 2>&1 \
      || { echo "run ex=$ex failed"; tail -20 "$O/exch_$ex.log"; exit 1; }
  python - "$O/exch_$ex.log" $ex <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("exchange", sys.argv[2], "every", d.get("exchange_every"), "ms_per_step", round(d["ms_per_step"], 4), "allgather_ms", d.get("allgather_ms"), "k2", d["kernels_ms"])
PY
done
echo done
