set -u
O=gpurun_out; mkdir -p $O
for lib in ${SCAN_LIBS:-metacov_amd/libmetacov_amd.so}; do
  for p in ${SCAN_PROCS:-base base,kmer,mirror,isize}; do
    METACOV_AMD_LIB=$lib timeout -k 10 200 python scripts/bench_scan.py --reads ${SCAN_READS:-100000000} --steps 5 --no-cpu-baseline --check 0 --procs $p > $O/r05t_scan.log 2>&1 || { echo "scan $lib $p failed"; tail -5 $O/r05t_scan.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['kernels_ms']['scan_kernel+kmer_count_kernel'],3))" $O/r05t_scan.log $(basename $lib) $p
  done
done
[ -n "${SKIP_C5:-}" ] && exit 0
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/r05t_bench_c5.log 2>&1 || { echo c5 failed; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['kernels_ms'])" $O/r05t_bench_c5.log
