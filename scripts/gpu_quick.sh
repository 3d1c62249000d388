#!/bin/bash
# GPU parity tests + prepare probe + default bench, each under its own limit;
# the first fatal status (fault / abort / timeout) ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-q}
O=$R/gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/${TAG}_pytest_gpu.log 2>&1
s=$?; tail -4 $O/${TAG}_pytest_gpu.log; [ $s -ne 0 ] && exit $s
fi
timeout -k 10 200 python scripts/prep_probe.py --config c3 > $O/${TAG}_prep.log 2>&1 || exit $?
timeout -k 10 200 python scripts/prep_probe.py --config c5 --reps 5 >> $O/${TAG}_prep.log 2>&1 || exit $?
grep prepare $O/${TAG}_prep.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/${TAG}_bench.log 2>&1 || { tail -5 $O/${TAG}_bench.log; exit 1; }
python - "$O/${TAG}_bench.log" <<'PY'
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print('value %.4g  ms/step %.4f  K2 %.4f  frac %.3f  prep %s' % (d['value'], d['ms_per_step'], d['kernels_ms'].get('k2_depth_fused_stats', d['kernels_ms'].get('k2_depth', 0)), d['roofline']['frac'], d.get('with_prepare')))
PY
