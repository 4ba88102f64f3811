#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile.  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r}
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 20 --no-cpu-baseline --no-ess > "$R/gpurun_out/${TAG}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${TAG}_prof.log"; exit 1; }
find "$R/gpurun_out/${TAG}_prof" -name "*stats*" | head
