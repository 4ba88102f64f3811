#!/bin/bash
# A/B of lane-resident kernel variants on the bench workload after the
# lane / parity tests: each argument after the tag and test list is an
# environment assignment list ("MC_LANES_FORM=0", "MC_LANES_FAST=0", "-" for
# the default).  Every GPU step has its own time limit.
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
for v in "$@"; do
  i=$((i+1))
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/${TAG}_bench_$i.json 2> gpurun_out/${TAG}_bench_$i.err || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_bench_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_bench_$i.json')); print('$v', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4), d['roofline']['kernel'])
"
done
