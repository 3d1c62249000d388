#!/bin/bash
# GPU tests on the box (prebuilt in-tree .so): pytest -m gpu over $TESTS
# (default: all), one process, each test under the thread timeout; a fatal
# status (fault / abort / timeout) ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05}
O=$R/gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout ${PER_TEST:-300} \
  --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > $O/${TAG}_pytest_gpu.log 2>&1
s=$?
grep -E "passed|failed|error" $O/${TAG}_pytest_gpu.log | tail -15
if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" $O/${TAG}_pytest_gpu.log; then echo "GPU fault"; exit 90; fi
exit $s
