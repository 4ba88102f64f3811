#!/bin/bash
# Headline bench at several slice counts (same binary, one box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-sp}
shift
for s in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess --slices $s > gpurun_out/${TAG}_s$s.json 2> gpurun_out/${TAG}_s$s.err || { echo "bench S=$s failed"; tail -3 gpurun_out/${TAG}_s$s.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${TAG}_s$s.json')); print('S=$s', round(d['value']/1e6,2), 'M', d['roofline']['frac'], d['roofline'].get('kernel'))"
done
