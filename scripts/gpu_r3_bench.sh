#!/bin/bash
# Bench lines on the current build: driver flags, default, small and medium
# shapes (each under its own limit; stop at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r3}
run() {  # name, limit, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { echo "bench $n failed"; tail -20 gpurun_out/${TAG}_$n.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${TAG}_$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,2), 'M steps/s frac', round(r['frac'],4), 'launch_ms', round(r['launch_ms'],4), 'ipl', r['iters_per_launch'], 'ess', d.get('ess_per_sec'), d.get('ess_timed',{}).get('ess_null_reason'), 'conv', (d.get('ess_converged') or {}).get('ess_per_sec'), (d.get('ess_converged') or {}).get('rhat'))"
}
run driver 300 --gpus 1 --steps 20 --warmup 5
run default 400
run small 300 --shape small --no-cpu-baseline
run medium 300 --shape medium --no-cpu-baseline
