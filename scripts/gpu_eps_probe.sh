#!/bin/bash
# Per-iteration kernel time of the driver's flags at several initial step sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-ep}
i=0
for e in 0 100 300 1000; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --clock-warm-ms $e --no-cpu-baseline --no-ess > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); print('$e', round(d['value']/1e6,2), 'M steps/s', 'per-iter', round(d['roofline']['kernel_ms']*1e3,2), 'us', 'acc', round(d['accept_rate'],3))
"
done
