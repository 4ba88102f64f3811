#!/bin/bash
# Round session: all GPU tests, the default bench (with CPU baseline), a
# kernel-trace profile of the bench and the two PMC traffic passes.  Every
# GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-full}
bash scripts/gpu_tests.sh ${TAG} tests > gpurun_out/${TAG}_tests_summary.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests_summary.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests_summary.log
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
bash scripts/gpu_profile.sh ${TAG}_prof || exit 1
