#!/bin/bash
# A/B of library builds on the bench workload (same box) after GPU tests:
# arguments after the tag and the test list are library paths ("-": the
# in-tree build).  Every GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; shift
TESTS=$1; shift
if [ "$TESTS" != "-" ]; then
timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
fi
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --steps 200 --warmup 50 > gpurun_out/${TAG}_bench_$i.json 2> gpurun_out/${TAG}_bench_$i.err || { echo "bench $lib failed"; tail -20 gpurun_out/${TAG}_bench_$i.err; exit 1; }
  else
    timeout -k 10 300 python scripts/ab_lib.py $lib --no-cpu-baseline --no-ess --steps 200 --warmup 50 > gpurun_out/${TAG}_bench_$i.json 2> gpurun_out/${TAG}_bench_$i.err || { echo "bench $lib failed"; tail -20 gpurun_out/${TAG}_bench_$i.err; exit 1; }
  fi
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_bench_$i.json')); print('$lib', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
done
