#!/bin/bash
# Sliced-kernel GPU session: its tests, then (unless the tests crashed or
# timed out) a bench run.  Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-sl}
timeout -k 10 600 python -m pytest tests/test_gpu_sliced.py -q -x > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -30 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
timeout -k 10 400 python bench.py --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
