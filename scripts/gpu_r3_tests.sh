#!/bin/bash
# Round-3 GPU session: the new parity tests, then bench lines (default,
# driver flags, small / medium shapes).  Every GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r3b}
shift
TESTS=${@:-tests/test_gpu_iso_parity.py tests/test_gpu_nuts_trace.py tests/test_gpu_multirank.py}
timeout -k 10 600 python -u -m pytest $TESTS -v -s -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error|near-tie|identical" gpurun_out/${TAG}_tests.log | head -40; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "identical|near-tie|agree|PASSED|two ranks" gpurun_out/${TAG}_tests.log | head -60
tail -1 gpurun_out/${TAG}_tests.log
