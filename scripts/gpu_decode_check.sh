set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_parity.py -k "decode or cli" -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gd_pytest.log 2>&1
s=$?; tail -25 gpurun_out/gd_pytest.log; if grep -qiE "memory access fault|illegal" gpurun_out/gd_pytest.log; then exit 90; fi
[ $s -gt 1 ] && exit $s
mkdir -p /tmp/e2e
timeout -k 10 400 python scripts/e2e.py --reads 30000000 --contigs 1000 --length 1000000 --dir /tmp/e2e > gpurun_out/gd_e2e.json 2> gpurun_out/gd_e2e.err
s=$?; tail -3 gpurun_out/gd_e2e.err; cat gpurun_out/gd_e2e.json; exit $s
