#!/bin/bash
# A/B of library builds over bench shapes (same box, alternating):
#   gpu_ab_shapes.sh TAG "SHAPE[:SLICES] ..." LIB...   ("-": the in-tree build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; SHAPES=$2; shift 2
for spec in $SHAPES; do
  sh=${spec%%:*}; sl=0
  [ "$spec" != "$sh" ] && sl=${spec#*:}
  i=0
  for lib in "$@"; do
    i=$((i+1))
    out=gpurun_out/${TAG}_${sh}_${sl}_$i
    if [ "$lib" = "-" ]; then
      timeout -k 10 300 python bench.py --shape $sh --slices $sl --no-cpu-baseline --no-ess --steps 200 --warmup 50 > $out.json 2> $out.err || { echo "bench $sh $lib failed"; tail -20 $out.err; exit 1; }
    else
      timeout -k 10 300 python scripts/ab_lib.py $lib --shape $sh --slices $sl --no-cpu-baseline --no-ess --steps 200 --warmup 50 > $out.json 2> $out.err || { echo "bench $sh $lib failed"; tail -20 $out.err; exit 1; }
    fi
    python -c "
import json
d=json.load(open('$out.json')); print('$sh:$sl $lib', round(d['value']/1e6,2), 'M steps/s', 'frac', round(d['roofline']['frac'],4), 'acc', round(d['accept_rate'],4))
"
  done
done
