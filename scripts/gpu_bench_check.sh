#!/bin/bash
# Bench lines under the driver's flags (twice) and defaults, then the
# multi-rank bench tests.  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-bc}
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_driver$i.json 2> gpurun_out/${TAG}_driver$i.err || { echo "bench (driver flags) failed"; tail -20 gpurun_out/${TAG}_driver$i.err; exit 1; }
  cut -c1-400 gpurun_out/${TAG}_driver$i.json
done
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_mr.log 2>&1 || { echo "multirank failed"; tail -20 gpurun_out/${TAG}_mr.log; exit 1; }
tail -1 gpurun_out/${TAG}_mr.log
