#!/bin/bash
# Per-launch HIP-event times under the driver's flags vs warmup length, launch
# size and launch kind.  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-lp}
i=0
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 100" "--steps 20 --warmup 500" "--steps 100 --warmup 5 --iters-per-launch 20" "--steps 20 --warmup 5 --iters-per-launch 5" "--steps 20 --warmup 5 --iters-per-launch 1" "COOP0 --steps 20 --warmup 5" "COOP0 --steps 100 --warmup 5 --iters-per-launch 20"; do
  i=$((i+1))
  E=""
  case "$a" in COOP0*) E="MC_COOPERATIVE=0"; a=${a#COOP0 };; esac
  timeout -k 10 200 env $E python bench.py $a --no-cpu-baseline --no-ess > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); r=d['roofline']; print('$E $a', round(d['value']/1e6,2), 'M', 'per-iter', round(r['kernel_ms']*1e3,2), 'us', 'each', r['each_launch_ms'])
"
done
