#!/bin/bash
# GPU decode / CLI parity tests, then the end-to-end timing (scripts/e2e.py); each step under its own limit.
mkdir -p gpurun_out /tmp/e2e
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "decode or cli" > gpurun_out/${TAG:-r03se}_pytest.log 2>&1
s=$?; grep -E "passed|failed|error" gpurun_out/${TAG:-r03se}_pytest.log | tail -5; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python scripts/e2e.py --reads 30000000 --contigs 1000 --length 1000000 --dir /tmp/e2e > gpurun_out/${TAG:-r03se}_e2e.json 2> gpurun_out/${TAG:-r03se}_e2e.err
s=$?; tail -3 gpurun_out/${TAG:-r03se}_e2e.err; python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['gpu_decode_s'],d['gpu_end_to_end_s'],d['gpu_decode_timings'])" gpurun_out/${TAG:-r03se}_e2e.json; exit $s
