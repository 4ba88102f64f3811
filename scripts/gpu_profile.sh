#!/bin/bash
# Profiles of the bench workload for profiles/: kernel-trace stats (timing)
# and two PMC passes (FETCH_SIZE, WRITE_SIZE) -> profiles/pmc_traffic.json.
# Every run uses bench.py's default launch size (50 iterations per launch;
# 50 warmup + 100 timed iterations = 3 full launches), so per-launch averages
# match the bench line's launch_ms / traffic.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 100 --warmup 50 --iters-per-launch 50 --no-cpu-baseline --no-ess"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_kt" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_kt.log" 2>&1 || { echo "kernel trace failed"; tail -20 "$R/gpurun_out/${TAG}_kt.log"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || { echo "fetch pass failed"; tail -20 "$R/gpurun_out/${TAG}_fetch.log"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/${TAG}_write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_write.log" 2>&1 || { echo "write pass failed"; tail -20 "$R/gpurun_out/${TAG}_write.log"; exit 1; }
cd "$R"
python3 scripts/pmc_traffic.py "gpurun_out/${TAG}_fetch" "gpurun_out/${TAG}_write" large 50
cp profiles/pmc_traffic.json gpurun_out/${TAG}_pmc_traffic.json
find "gpurun_out/${TAG}_kt" -name "*kernel_stats*"
