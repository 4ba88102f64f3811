#!/bin/bash
# Kernel traces of the final build: the default bench launch size (50
# iterations, clocks warmed by bf16 GEMMs so every sampler dispatch is a
# timed-size launch) and the driver's flags (--steps 20 --warmup 5).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-v43}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${TAG}_kt -o run -- python3 "$R/bench.py" --steps 1000 --warmup 500 --iters-per-launch 50 --no-cpu-baseline --no-ess --clock-warm-kind gemm --clock-warm-ms 1000 > "$R/gpurun_out/${TAG}_kt.log" 2>&1 || { echo "kt failed"; exit 1; }
python3 "$R/scripts/prof_filter.py" /tmp/prof_${TAG}_kt "$R/gpurun_out/${TAG}_kt" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${TAG}_kt20 -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-ess > "$R/gpurun_out/${TAG}_kt20.log" 2>&1 || { echo "kt20 failed"; exit 1; }
python3 "$R/scripts/prof_filter.py" /tmp/prof_${TAG}_kt20 "$R/gpurun_out/${TAG}_kt20" || exit 1
echo kt done
