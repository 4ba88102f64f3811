#!/bin/bash
# A/B of an environment switch of the library on the README small / medium /
# large shapes, alternating on one box:  gpu_env_ab.sh TAG VAR VALUE [shapes]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; VAR=$2; VAL=$3; shift 3
SHAPES=${@:-small medium large}
for sh in $SHAPES; do
  for v in default $VAL default $VAL; do
    if [ "$v" = "default" ]; then unset $VAR; else export $VAR=$v; fi
    timeout -k 10 300 python bench.py --shape $sh --no-cpu-baseline --no-ess --steps 200 --warmup 50 > gpurun_out/${TAG}_${sh}_$v.json 2> gpurun_out/${TAG}_${sh}_$v.err || { echo "bench $sh $v failed"; tail -20 gpurun_out/${TAG}_${sh}_$v.err; exit 1; }
    python -c "
import json
d=json.load(open('gpurun_out/${TAG}_${sh}_$v.json')); print('$sh $VAR=$v', round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
  done
done
unset $VAR
