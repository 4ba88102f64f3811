#!/bin/bash
# NUTS parity tests on the in-tree build, then two config-5 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-nq}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_samplers.py tests/test_gpu_affine.py tests/test_gpu_kernel_note.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload nuts --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); print(round(d['value']/1e6,2), 'M leaves/s', 'depth', round(d['mean_tree_depth'],4), 'leaves', d['leaves'], 'acc', d['accept_stat_mean'], 'eps', d['step_size'])
"
done
