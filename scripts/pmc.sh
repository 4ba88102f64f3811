#!/bin/bash
# PMC passes over a short bench run (counters only; no tracing domains).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
shift
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters.txt" 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-ess > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/${TAG}_p$i.log"; exit 1; }
done
echo done
