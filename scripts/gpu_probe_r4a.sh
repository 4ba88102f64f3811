#!/bin/bash
# Round-4 probes: packed/scalar FP32 issue rates (scripts/micro/pk_probe) and
# the section stamps of k_hmc_lf at the large / medium / small shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r4p}
timeout -k 10 60 ./scripts/micro/pk_probe > gpurun_out/${TAG}_pk_probe.log 2>&1 || { echo "pk_probe failed"; tail gpurun_out/${TAG}_pk_probe.log; exit 1; }
cat gpurun_out/${TAG}_pk_probe.log
timeout -k 10 60 ./scripts/micro/rng_probe > gpurun_out/${TAG}_rng_probe.log 2>&1 || { echo "rng_probe failed"; tail gpurun_out/${TAG}_rng_probe.log; exit 1; }
cat gpurun_out/${TAG}_rng_probe.log
for sh in large medium small; do
  timeout -k 10 120 python -u scripts/stamps_lf.py $sh 256 > gpurun_out/${TAG}_stamps_$sh.log 2>&1 || { echo "stamps $sh failed"; tail -20 gpurun_out/${TAG}_stamps_$sh.log; exit 1; }
  cat gpurun_out/${TAG}_stamps_$sh.log
done
timeout -k 10 120 python -u scripts/stamps_nuts.py > gpurun_out/${TAG}_stamps_nuts.log 2>&1 || { echo "stamps nuts failed"; tail -20 gpurun_out/${TAG}_stamps_nuts.log; exit 1; }
cat gpurun_out/${TAG}_stamps_nuts.log
