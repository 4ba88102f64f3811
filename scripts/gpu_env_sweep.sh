#!/bin/bash
# Sweep of an environment switch on one shape, two alternating rounds on one
# box:  gpu_env_sweep.sh TAG VAR SHAPE VALUES...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; VAR=$2; SH=$3; shift 3
for round in 1 2; do
  for v in "$@"; do
    export $VAR=$v
    timeout -k 10 300 python bench.py --shape $SH --no-cpu-baseline --no-ess --steps 200 --warmup 50 $BENCH_ARGS > gpurun_out/${TAG}_${SH}_${v}_$round.json 2> gpurun_out/${TAG}_${SH}_${v}_$round.err || { echo "bench $SH $v failed"; tail -20 gpurun_out/${TAG}_${SH}_${v}_$round.err; exit 1; }
    python -c "
import json
d=json.load(open('gpurun_out/${TAG}_${SH}_${v}_$round.json')); print('$SH $VAR=$v', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
  done
done
unset $VAR
