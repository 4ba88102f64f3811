#!/bin/bash
# GPU tests only (optionally a subset: $2 = pytest path/args).  One time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-t}
SEL=${2:-tests}
timeout -k 10 900 python -u -m pytest $SEL -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -40
if [ $rc -ne 0 ]; then grep -B5 -A40 "Error\|assert" gpurun_out/${TAG}_tests.log | head -120; fi
exit $rc
