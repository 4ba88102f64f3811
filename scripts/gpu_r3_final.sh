#!/bin/bash
# Round-3 final pass on one box: the whole GPU suite, smoke(), the default
# bench line, the driver's flags and the expression-throughput probe.  Every
# GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-v29}
bash scripts/gpu_r3c.sh "$TAG" || exit 1
timeout -k 10 240 python -u scripts/bench_expr.py > gpurun_out/${TAG}_bench_expr.log 2>&1 || { echo "bench_expr failed"; tail -5 gpurun_out/${TAG}_bench_expr.log; exit 1; }
tail -4 gpurun_out/${TAG}_bench_expr.log
