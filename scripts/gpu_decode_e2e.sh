mkdir -p gpurun_out /tmp/e2e
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "decode or cli" > gpurun_out/r03se_pytest.log 2>&1
s=$?; grep -E "passed|failed|error" gpurun_out/r03se_pytest.log | tail -5; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python scripts/e2e.py --reads 30000000 --contigs 1000 --length 1000000 --dir /tmp/e2e --gpu-windows 4096 > gpurun_out/r03se_e2e.json 2> gpurun_out/r03se_e2e.err
s=$?; tail -3 gpurun_out/r03se_e2e.err; python -c "import json;d=json.load(open('gpurun_out/r03se_e2e.json'));print(d['gpu_decode_s'],d['gpu_end_to_end_s'],d['gpu_decode_timings'])"; exit $s
