#!/bin/bash
# Soak run of the direct / full-prepare fuzz (tests/test_gpu_parity.py::
# test_direct_and_full_fuzz) over several seeds; one pytest process per seed,
# each under its own limit; the first failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
for seed in ${SEEDS:-11 12 13 14 15 16}; do
  MC_FUZZ_SEED=$seed MC_FUZZ_ITERS=${ITERS:-40} timeout -k 10 170 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      -k test_direct_and_full_fuzz --timeout 160 --timeout-method thread --durations=1 > "$O/soak_$seed.log" 2>&1 \
      || { echo "seed $seed failed"; tail -30 "$O/soak_$seed.log"; exit 1; }
  echo "seed $seed: $(grep -E 'passed|failed' $O/soak_$seed.log | tail -1)"
done
echo done
