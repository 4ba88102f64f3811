#!/bin/bash
# Round-4 profiles of the bench workload: kernel traces at the default launch
# size (50 iterations) and at the driver's (--steps 20: one 20-iteration
# launch), FETCH / WRITE passes at both sizes, two SQ passes, the small /
# medium shapes' kernel traces and the NUTS line's (no clock warm: every
# dispatch of the sampler kernel has the profiled size).  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r4p}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
A50="--steps 100 --warmup 50 --iters-per-launch 50 --no-cpu-baseline --no-ess --clock-warm-ms 0"
A20="--steps 20 --warmup 20 --no-cpu-baseline --no-ess --clock-warm-ms 0"
# kernel traces: warm clocks from bf16 GEMMs (another kernel, so every
# sampler dispatch in the trace is a timed-size launch) and a long run
K50="--steps 1000 --warmup 500 --iters-per-launch 50 --no-cpu-baseline --no-ess --clock-warm-kind gemm --clock-warm-ms 1000"
K20="--steps 20 --warmup 20 --no-cpu-baseline --no-ess --clock-warm-kind gemm --clock-warm-ms 1000"
run() {  # name, bench args (quoted), rocprof args...
  local n=$1 args=$2; shift 2
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "/tmp/prof_${TAG}_$n" -o run -- python3 "$R/bench.py" $args > "$R/gpurun_out/${TAG}_$n.log" 2>&1 || { echo "$n failed rc=$?"; grep -v "^ *@" "$R/gpurun_out/${TAG}_$n.log" | tail -5; exit 1; }
  python3 "$R/scripts/prof_filter.py" "/tmp/prof_${TAG}_$n" "$R/gpurun_out/${TAG}_$n" && rm -rf "/tmp/prof_${TAG}_$n"
}
run kt "$K50" --kernel-trace --stats
run kt20 "$K20" --kernel-trace --stats
run fetch "$A50" --pmc FETCH_SIZE
run write "$A50" --pmc WRITE_SIZE
run fetch20 "$A20" --pmc FETCH_SIZE
run write20 "$A20" --pmc WRITE_SIZE
run sq1 "$A50" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM
run sq2 "$A50" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU
run kt_small "--shape small $K50" --kernel-trace --stats
run kt_medium "--shape medium $K50" --kernel-trace --stats
run kt_nuts "--workload nuts --steps 200 --warmup 200 --iters-per-launch 50 --no-cpu-baseline" --kernel-trace --stats
echo profiles done
