#!/bin/bash
# One GPU session: the GPU test suite, the bench under the driver's flags and
# with defaults, then the rocprof kernel trace of the bench workload.  Every
# GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-s}
bash scripts/gpu_r2.sh "$TAG" "${2:-tests}" || exit 1
bash scripts/gpu_profile.sh "$TAG" || exit 1
