#!/bin/bash
# Stamps (per-section cycles) and two SQ counter passes of the bench
# workload (plain launches: the cooperative launch's teardown crashes under
# rocprofv3 at exit).  Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sq}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 120 python scripts/stamps_lr.py 256 > gpurun_out/${TAG}_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/${TAG}_stamps.log; exit 1; }
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 100 --warmup 50 --iters-per-launch 50 --no-cpu-baseline --no-ess"
run() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$R/gpurun_out/${TAG}_$n" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_$n.log" 2>&1 || { echo "$n failed rc=$?"; grep -v "^ *@" "$R/gpurun_out/${TAG}_$n.log" | tail -5; exit 1; }
}
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM
run sq2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU
echo pmc done
