#!/bin/bash
# A/B of the lane-resident kernels on the bench workload (MC_LANES_FAST=0:
# k_hmc_lr; default: k_hmc_lf for fast-form programs), after the sliced and
# parity tests.  Every GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-ab}
TESTS=${2:-"tests/test_gpu_sliced.py tests/test_gpu_large_parity.py tests/test_gpu_posterior_parity.py"}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for v in 1 0 1; do
  MC_LANES_FAST=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/${TAG}_bench_$v.json 2> gpurun_out/${TAG}_bench_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_bench_$v.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_bench_$v.json')); print('fast=$v', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
done
