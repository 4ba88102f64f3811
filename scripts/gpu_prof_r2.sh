#!/bin/bash
# Round-2 profiles of the bench workload with plain (non-cooperative) launches:
# under rocprofv3 the cooperative launch's teardown crashes the process at
# exit (after the profiler has written its files).  Kernel trace, FETCH/WRITE
# passes and two SQ passes.  Each GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2p}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 100 --warmup 50 --iters-per-launch 50 --no-cpu-baseline --no-ess"
run() {  # name, rocprof args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$R/gpurun_out/${TAG}_$n" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_$n.log" 2>&1 || { echo "$n failed rc=$?"; grep -v "^ *@" "$R/gpurun_out/${TAG}_$n.log" | tail -5; exit 1; }
}
NARGS="--workload nuts --steps 200 --warmup 200 --iters-per-launch 50 --no-cpu-baseline"
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM
run sq2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_nuts_kt" -o run -- python3 "$R/bench.py" $NARGS > "$R/gpurun_out/${TAG}_nuts_kt.log" 2>&1 || { echo "nuts kt failed"; exit 1; }
echo profiles done
