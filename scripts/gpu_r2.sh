#!/bin/bash
# Round-2 GPU session: parity tests (the large-shape oracle trace first), the
# bench under the driver's flags and with defaults.  Every GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r2}
SEL=${2:-tests}
timeout -k 10 600 python -u -m pytest $SEL -v -m gpu -x --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.json 2> gpurun_out/${TAG}_bench_driver.err || { echo "bench (driver flags) failed"; tail -30 gpurun_out/${TAG}_bench_driver.err; exit 1; }
cat gpurun_out/${TAG}_bench_driver.json
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
