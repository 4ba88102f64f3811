#!/bin/bash
# A/B of the replicated lane layout (MC_LANES_REP=1: off) on the README
# small / medium / large shapes, alternating on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-rep}
for sh in small medium large; do
  for v in default 1 default 1; do
    if [ "$v" = "default" ]; then unset MC_LANES_REP; else export MC_LANES_REP=$v; fi
    timeout -k 10 300 python bench.py --shape $sh --no-cpu-baseline --no-ess --steps 200 --warmup 50 > gpurun_out/${TAG}_${sh}_$v.json 2> gpurun_out/${TAG}_${sh}_$v.err || { echo "bench $sh $v failed"; tail -20 gpurun_out/${TAG}_${sh}_$v.err; exit 1; }
    python -c "
import json
d=json.load(open('gpurun_out/${TAG}_${sh}_$v.json')); print('$sh rep=$v', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
  done
done
unset MC_LANES_REP
