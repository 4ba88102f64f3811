#!/bin/bash
# Bench one shape at several slice counts (0: automatic):
#   gpu_slices_r4.sh TAG SHAPE "0 8 16" [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; SH=$2; LIST=$3; shift 3
for a in $LIST; do
  timeout -k 10 300 python bench.py --shape $SH --no-cpu-baseline --no-ess --steps 200 --warmup 50 --slices $a "$@" > gpurun_out/${TAG}_${SH}_$a.json 2> gpurun_out/${TAG}_${SH}_$a.err || { echo "bench $a failed"; tail -20 gpurun_out/${TAG}_${SH}_$a.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_${SH}_$a.json')); c=d['config']; print('$SH slices=$a', c.get('slices'), c.get('kernel'), round(d['value']/1e6,2), 'M steps/s', 'launch_ms', round(d['roofline']['launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
done
