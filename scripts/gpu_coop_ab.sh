#!/bin/bash
# Cooperative vs plain launches of the bench kernel: 8 launches of 20
# iterations each, alternating, three rounds on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-co}
i=0
for r in 1 2 3; do for c in 1 0; do
  i=$((i+1))
  MC_COOPERATIVE=$c timeout -k 10 200 python bench.py --steps 160 --warmup 20 --iters-per-launch 20 --no-cpu-baseline --no-ess > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); r=d['roofline']; print('coop=$c', round(d['value']/1e6,2), 'M', 'each', r['each_launch_ms'])
"
done; done
