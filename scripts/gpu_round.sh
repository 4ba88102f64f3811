#!/bin/bash
# GPU session steps (run through gpurun from the repo root).  Every GPU step
# has its own time limit; `all`-style chains stop at the first failure.
#
#   bash scripts/gpu_round.sh tests TAG [pytest args...]   GPU tests (default: all -m gpu)
#   bash scripts/gpu_round.sh smoke TAG                    __graft_entry__.smoke()
#   bash scripts/gpu_round.sh bench TAG NAME [bench args]  one bench line -> TAG_bench_NAME.json
#   bench-lines TAG                                        the round's bench lines: default,
#                                                          driver flags, small, medium, NUTS
#                                                          config 5 and Large
#   bash scripts/gpu_round.sh kt TAG NAME [bench args]     rocprofv3 kernel trace + stats of a
#                                                          bench run (filtered: prof_filter.py)
#   bash scripts/gpu_round.sh pmc TAG NAME KERNEL IPL L FLOOR KEY [bench args]
#                                                          FETCH / WRITE passes and the two SQ
#                                                          passes (separate runs), SQ summary
#                                                          of KERNEL (pmc_sq.py) per wave-step
#                                                          of IPL-iteration launches of L steps
#                                                          (every dispatch of KERNEL in the run
#                                                          must be one: --clock-warm-kind gemm
#                                                          --no-ess, warmup/steps multiples of
#                                                          --iters-per-launch); FLOOR = the
#                                                          sweep's VALU per wave-step (0: none);
#                                                          the HBM bytes per launch go to
#                                                          gpurun_out/TAG_traffic.json under
#                                                          KEY@IPL (bench.py pmc_traffic)
#   bash scripts/gpu_round.sh traffic TAG NAME KERNEL IPL KEY [bench args]
#                                                          the FETCH / WRITE passes only: the
#                                                          traffic record KEY@IPL
#   bash scripts/gpu_round.sh ab TAG LIB... [-- bench args] A/B of library builds on one box
#                                                          ("-" = the in-tree build)
#   bash scripts/gpu_round.sh final TAG                    tests + smoke + bench-lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEP=$1; TAG=$2; shift 2
export TMPDIR=/tmp

tests() {
  local sel=("$@")
  [ ${#sel[@]} -eq 0 ] && sel=(tests)
  timeout -k 10 1100 python -u -m pytest "${sel[@]}" -v -m gpu -x --timeout 180 \
      --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
    || { echo "tests failed"; grep -E "^E |FAILED|Error|passed|failed" gpurun_out/${TAG}_tests.log | head -40; tail -5 gpurun_out/${TAG}_tests.log; return 1; }
  tail -2 gpurun_out/${TAG}_tests.log
}

smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.build.__doc__; g.smoke(); print('smoke ok')" \
      > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; return 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
}

bench() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${TAG}_bench_$n.json \
      2> gpurun_out/${TAG}_bench_$n.err || { echo "bench $n failed"; tail -20 gpurun_out/${TAG}_bench_$n.err; return 1; }
  python -c "
import json
d = json.load(open('gpurun_out/${TAG}_bench_$n.json'))
r = d.get('roofline', {})
print('$n', round(d['value'] / 1e6, 3), 'M', d['unit'], 'frac', round(r.get('frac', 0), 4),
      'launch_ms', round(r.get('launch_ms', 0), 4), r.get('kernel', ''))
"
}

bench_lines() {
  bench default || return 1
  bench driver --steps 20 --warmup 5 || return 1
  bench small --shape small --no-cpu-baseline || return 1
  bench medium --shape medium --no-cpu-baseline || return 1
  bench nuts --workload nuts || return 1
  bench nuts_large --workload nuts --nuts-model hier --shape large --chains 256 --steps 20 --warmup 20 || return 1
}

prof() {  # name, bench args (one string), rocprof args...
  local n=$1 args=$2; shift 2
  (cd /tmp && timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "/tmp/prof_${TAG}_$n" -o run \
      -- python3 "$R/bench.py" $args > "$R/gpurun_out/${TAG}_$n.log" 2>&1) \
    || { echo "$n failed rc=$?"; grep -v "^ *@" "$R/gpurun_out/${TAG}_$n.log" | tail -5; return 1; }
  python3 "$R/scripts/prof_filter.py" "/tmp/prof_${TAG}_$n" "$R/gpurun_out/${TAG}_$n" && rm -rf "/tmp/prof_${TAG}_$n"
}

case $STEP in
  tests) tests "$@" ;;
  smoke) smoke ;;
  bench) bench "$@" ;;
  bench-lines) bench_lines ;;
  kt) n=$1; shift; prof kt_$n "$*" --kernel-trace --stats ;;
  sq1)  # NAME [bench args]: the instruction-mix SQ pass alone
    n=$1; shift
    prof sq1_$n "$*" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM ;;
  pmc)
    n=$1; k=$2; ipl=$3; lf=$4; fl=$5; key=$6; shift 6
    prof fetch_$n "$*" --pmc FETCH_SIZE && prof write_$n "$*" --pmc WRITE_SIZE &&
    prof sq1_$n "$*" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM &&
    prof sq2_$n "$*" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU &&
    python scripts/pmc_sq.py gpurun_out/${TAG}_sq_$n.json "$k" "$ipl" "$lf" --floor "$fl" gpurun_out/${TAG}_sq1_$n gpurun_out/${TAG}_sq2_$n &&
    python scripts/pmc_traffic.py gpurun_out/${TAG}_fetch_$n gpurun_out/${TAG}_write_$n "$key" "$ipl" \
        "profiles/$TAG: fetch_$n|write_$n (bench.py $*)" --kernel "$k" --out gpurun_out/${TAG}_traffic.json ;;
  traffic)  # NAME KERNEL IPL KEY [bench args]: the FETCH / WRITE passes and the traffic record
    n=$1; k=$2; ipl=$3; key=$4; shift 4
    prof fetch_$n "$*" --pmc FETCH_SIZE && prof write_$n "$*" --pmc WRITE_SIZE &&
    python scripts/pmc_traffic.py gpurun_out/${TAG}_fetch_$n gpurun_out/${TAG}_write_$n "$key" "$ipl" \
        "profiles/$TAG: fetch_$n|write_$n (bench.py $*)" --kernel "$k" --out gpurun_out/${TAG}_traffic.json ;;
  ab)
    libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    i=0
    for lib in "${libs[@]}"; do
      i=$((i+1))
      if [ "$lib" = "-" ]; then
        timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess "$@" > gpurun_out/${TAG}_ab_$i.json 2> gpurun_out/${TAG}_ab_$i.err || { echo "bench $lib failed"; tail -20 gpurun_out/${TAG}_ab_$i.err; exit 1; }
      else
        timeout -k 10 300 python scripts/ab_lib.py "$lib" --no-cpu-baseline --no-ess "$@" > gpurun_out/${TAG}_ab_$i.json 2> gpurun_out/${TAG}_ab_$i.err || { echo "bench $lib failed"; tail -20 gpurun_out/${TAG}_ab_$i.err; exit 1; }
      fi
      python -c "
import json
d = json.load(open('gpurun_out/${TAG}_ab_$i.json')); r = d['roofline']
print('$lib', round(d['value'] / 1e6, 3), 'M', 'launch_ms', round(r['launch_ms'], 4), 'frac', round(r['frac'], 4))
"
    done ;;
  final) tests && smoke && bench_lines ;;
  *) echo "unknown step $STEP"; exit 2 ;;
esac
