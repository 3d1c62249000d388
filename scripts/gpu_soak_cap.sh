#!/bin/bash
# Soak run of tests/test_depth_cap.py::test_device_cap_mask_random_sets over
# several seeds (one pytest process per seed, each under its own limit).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
for seed in ${SEEDS:-1 2 3 4}; do
  MC_CAP_SOAK_SEED=$seed MC_CAP_SOAK_ITERS=${ITERS:-100} timeout -k 10 170 python -u -m pytest tests/test_depth_cap.py -m gpu -x -q \
      -k test_device_cap_mask_random_sets --timeout 160 --timeout-method thread > "$O/soakcap_$seed.log" 2>&1 \
      || { echo "seed $seed failed"; tail -30 "$O/soakcap_$seed.log"; exit 1; }
  echo "seed $seed: $(grep -E 'passed|failed' $O/soakcap_$seed.log | tail -1)"
done
echo done
