#!/bin/bash
# Bench at the automatic slice count and at 8 slices (4 waves per CU), twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-sl}
for a in "0" "8" "0" "8"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --steps 200 --warmup 50 --slices $a > gpurun_out/${TAG}_$a.json 2> gpurun_out/${TAG}_$a.err || { echo "bench $a failed"; tail -20 gpurun_out/${TAG}_$a.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$a.json')); print('slices=$a', d['config']['slices'], round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
done
