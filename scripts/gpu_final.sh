#!/bin/bash
# Round-end GPU session on the current build: every GPU test, smoke(), the
# bench under the driver's flags and with defaults, the config-5 NUTS line,
# then the kernel-trace / PMC profiles (gpu_prof_r2.sh).  Every GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-fin}
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.json 2> gpurun_out/${TAG}_bench_driver.err || { echo "bench (driver flags) failed"; tail -30 gpurun_out/${TAG}_bench_driver.err; exit 1; }
cat gpurun_out/${TAG}_bench_driver.json
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python bench.py --workload nuts > gpurun_out/${TAG}_nuts_bench.json 2> gpurun_out/${TAG}_nuts_bench.err || { echo "nuts bench failed"; tail -5 gpurun_out/${TAG}_nuts_bench.err; exit 1; }
cat gpurun_out/${TAG}_nuts_bench.json
bash scripts/gpu_prof_r2.sh ${TAG}p || exit 1
