#!/bin/bash
# Per-launch overhead A/B under the driver's flags (--steps 20 --warmup 5):
# in-tree build vs scripts/libmcmc355_prev.so, cooperative vs plain launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-la}
i=0
for v in "-" "MC_COOPERATIVE=0" "PREV" "-"; do
  i=$((i+1))
  if [ "$v" = "PREV" ]; then
    timeout -k 10 200 python scripts/ab_lib.py scripts/libmcmc355_prev.so --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  else
    [ "$v" = "-" ] && v=""
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  fi
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); print('$v', round(d['value']/1e6,2), 'M steps/s', 'ms/step', round(d['ms_per_step'],4), 'launch_ms', round(d['roofline']['launch_ms'],4))
"
done
