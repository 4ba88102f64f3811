#!/bin/bash
# Two SQ counter passes of the config-5 NUTS bench (k_nuts_lr).  Each GPU
# step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-nsq}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
ARGS="--workload nuts --steps 100 --warmup 100 --iters-per-launch 50 --no-cpu-baseline"
run() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "/tmp/prof_${TAG}_$n" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_$n.log" 2>&1 || { echo "$n failed rc=$?"; grep -v "^ *@" "$R/gpurun_out/${TAG}_$n.log" | tail -5; exit 1; }
  python3 "$R/scripts/prof_filter.py" "/tmp/prof_${TAG}_$n" "$R/gpurun_out/${TAG}_$n" && rm -rf "/tmp/prof_${TAG}_$n"
}
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM
run sq2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU
run sq3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64
echo pmc done
