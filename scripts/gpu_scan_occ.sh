set -u
O=gpurun_out
TAG=r05zh TESTS="tests/test_scan.py" bash scripts/gpu_tests.sh || exit 1
SKIP_C5=1 SCAN_LIBS="metacov_amd/libmetacov_amd.so metacov_amd/variants/lib_occ3.so metacov_amd/variants/lib_r1024.so metacov_amd/variants/lib_s4864.so metacov_amd/libmetacov_amd.so metacov_amd/variants/lib_r1024.so" SCAN_PROCS="base,kmer,mirror,isize" bash scripts/gpu_scan_ab.sh > $O/r05zh_scan_occupancy.txt 2>&1 || exit 1
cat $O/r05zh_scan_occupancy.txt
timeout -k 10 300 python scripts/bench_scan.py --check 4000000 > $O/r05zh_scan_bench.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r05zh_scan_bench.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['cpu_baseline']['value'])"
