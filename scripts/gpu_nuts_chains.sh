#!/bin/bash
# NUTS (config 5 model) throughput vs chains per GPU: how far the 64-chain
# line is from the chip's capacity.  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-nc}
shift
for c in "$@"; do
  timeout -k 10 200 python bench.py --workload nuts --chains $c --no-cpu-baseline > gpurun_out/${TAG}_c$c.json 2> gpurun_out/${TAG}_c$c.err || { echo "nuts C=$c failed"; tail -3 gpurun_out/${TAG}_c$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${TAG}_c$c.json')); r=d['roofline']; print('C=$c', round(d['value']/1e6,2), 'M leaf-steps/s', 'frac', round(r['frac'],5), 'launch_ms', round(r['launch_ms'],3), 'depth', round(d['mean_tree_depth'],3), r['kernel'])"
done
