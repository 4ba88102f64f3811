#!/bin/bash
# Round-6 PMC records (run through gpurun): the SQ + traffic passes of the
# driver-size headline launch (20 iterations) and the traffic records of the
# other bench lines (profiles/pmc_traffic.json keys, bench.py pmc_traffic).
set -o pipefail
T=${1:-p6}
G="bash scripts/gpu_round.sh"
$G pmc $T large20 k_hmc_lf 20 20 293 large --steps 40 --warmup 20 --iters-per-launch 20 \
    --clock-warm-kind gemm --no-ess --no-cpu-baseline &&
$G traffic $T large50 k_hmc_lf 50 large --steps 100 --warmup 50 --clock-warm-kind gemm \
    --no-ess --no-cpu-baseline &&
$G traffic $T small k_hmc_lf 50 small --shape small --steps 100 --warmup 50 \
    --clock-warm-kind gemm --no-ess --no-cpu-baseline &&
$G traffic $T medium k_hmc_lf 50 medium --shape medium --steps 100 --warmup 50 \
    --clock-warm-kind gemm --no-ess --no-cpu-baseline &&
$G traffic $T nuts k_nuts_lr 50 nuts-illcond --workload nuts --steps 200 --warmup 100 \
    --no-cpu-baseline &&
$G traffic $T nuts_large k_nuts_sl 20 nuts-hier-large --workload nuts --nuts-model hier \
    --shape large --chains 256 --steps 20 --warmup 20 --no-cpu-baseline &&
$G traffic $T mh k_mh_sl 50 mh-large --workload mh --steps 200 --warmup 100 --no-cpu-baseline
