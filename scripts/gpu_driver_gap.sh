#!/bin/bash
# Where the driver-flag run (--steps 20 --warmup 5) loses against the default
# run: clock warm-up length vs launch length.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-dg}
i=0
while read -r args; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess $args > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "bench failed: $args"; tail -3 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); r=d['roofline']; print('$args |', round(d['value']/1e6,2), 'M', 'launch_ms', round(r.get('launch_ms',0),3), 'frac', round(r['frac'],4))"
done <<'LIST'
--steps 20 --warmup 5
--steps 20 --warmup 5 --clock-warm-ms 2000
--steps 20 --warmup 50
--steps 100 --warmup 5
--steps 20 --warmup 5 --iters-per-launch 10
--steps 1000 --warmup 500
LIST
