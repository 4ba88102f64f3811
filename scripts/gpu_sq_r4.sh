#!/bin/bash
# The two SQ counter passes of the bench workload (50-iteration launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r4sq}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
A50="--steps 100 --warmup 50 --iters-per-launch 50 --no-cpu-baseline --no-ess --clock-warm-ms 0 $EXTRA_ARGS"
run() {
  local n=$1 args=$2; shift 2
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "/tmp/prof_${TAG}_$n" -o run -- python3 "$R/bench.py" $args > "$R/gpurun_out/${TAG}_$n.log" 2>&1 || { echo "$n failed rc=$?"; grep -v "^ *@" "$R/gpurun_out/${TAG}_$n.log" | tail -5; exit 1; }
  python3 "$R/scripts/prof_filter.py" "/tmp/prof_${TAG}_$n" "$R/gpurun_out/${TAG}_$n" && rm -rf "/tmp/prof_${TAG}_$n"
}
run sq1 "$A50" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM
run sq2 "$A50" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU
cd "$R"
python scripts/pmc_sq.py gpurun_out/${TAG}.json k_hmc_lf 50 20 gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2 && cat gpurun_out/${TAG}.json
