#!/bin/bash
# NUTS A/B of library builds (config 5 line, same box, alternating), after
# the NUTS parity tests:  gpu_nuts_ab4.sh TAG LIB...   ("-": the in-tree build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_nuts_trace.py tests/test_gpu_parity.py -x -q -m gpu -k "nuts" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
i=0
for lib in "$@"; do
  i=$((i+1))
  out=gpurun_out/${TAG}_nuts_$i
  if [ "$lib" = "-" ]; then
    timeout -k 10 300 python bench.py --workload nuts --no-cpu-baseline --no-ess $NUTS_ARGS > $out.json 2> $out.err || { echo "bench $lib failed"; tail -20 $out.err; exit 1; }
  else
    timeout -k 10 300 python scripts/ab_lib.py $lib --workload nuts --no-cpu-baseline --no-ess $NUTS_ARGS > $out.json 2> $out.err || { echo "bench $lib failed"; tail -20 $out.err; exit 1; }
  fi
  python -c "
import json
d=json.load(open('$out.json')); print('$lib', round(d['value']/1e6,2), 'M leaf-steps/s', 'depth', d.get('mean_tree_depth', d.get('config',{}).get('mean_tree_depth')), 'ms', round(d['ms_per_step'],4))
"
done
