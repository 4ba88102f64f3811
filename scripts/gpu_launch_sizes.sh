#!/bin/bash
# Timed-iteration cost by launch size and start state (bench workload).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-ls}
i=0
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 500" "--steps 100 --warmup 5 --iters-per-launch 20" "--steps 100 --warmup 5" "--steps 200 --warmup 5 --iters-per-launch 200"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-ess > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); print('$a', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'per-iter', round(d['roofline']['kernel_ms']*1e3,2), 'us', 'eps', round(d['step_size'],6))
"
done
