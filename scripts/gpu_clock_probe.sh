#!/bin/bash
# Per-iteration kernel time under the driver's flags (--steps 20 --warmup 5)
# for several clock-warm kinds and lengths.  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-cp}
shift
LIST=("$@")
[ ${#LIST[@]} -eq 0 ] && LIST=("gemm 0" "gemm 500" "sampler 300" "gemm 2000" "sampler 1000" "gemm 500" "sampler 300")
i=0
for kw in "${LIST[@]}"; do
  set -- $kw
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --clock-warm-kind $1 --clock-warm-ms $2 --no-cpu-baseline --no-ess > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/${TAG}_$i.json')); print('$1 $2', round(d['value']/1e6,2), 'M steps/s', 'per-iter', round(d['roofline']['kernel_ms']*1e3,2), 'us', 'acc', d['accept_rate'], 'eps', d['step_size'])
"
done
