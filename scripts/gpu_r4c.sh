#!/bin/bash
# Round-4 pass: the whole GPU suite, the replication A/B (small / medium /
# large), the step-specialisation A/B against the round-3 k_hmc_lf, section
# stamps and the expression / affine throughput probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r4c}
EXPR=1 bash scripts/gpu_r4.sh $TAG all || exit 1
bash scripts/gpu_rep_ab.sh ${TAG}rep || exit 1
bash scripts/gpu_ablib.sh ${TAG}ab - - scripts/_tmp_lib_r3lf.so - scripts/_tmp_lib_r3lf.so || exit 1
bash scripts/gpu_probe_r4a.sh ${TAG}p || exit 1
