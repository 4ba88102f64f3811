#!/bin/bash
# NUTS tests, then config-5 bench lines: in-tree build vs scripts/libmcmc355_prev.so.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-na}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_samplers.py tests/test_gpu_multirank.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
i=0
for lib in - scripts/libmcmc355_prev.so - scripts/libmcmc355_prev.so; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then
    timeout -k 10 200 python bench.py --workload nuts --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "bench failed"; exit 1; }
  else
    timeout -k 10 200 python scripts/ab_lib.py $lib --workload nuts --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "bench failed"; exit 1; }
  fi
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); print('$lib', round(d['value']/1e6,2), 'M leaves/s', 'depth', round(d['mean_tree_depth'],3))
"
done
