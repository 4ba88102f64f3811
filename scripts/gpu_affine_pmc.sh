#!/bin/bash
# SQ counters of the chain-per-workgroup tape on the N = 100 K regression
# (fused affine term and the hand-written expression).  One pass each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for w in fused expr; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/aff_${w}_kt" -o run -- python3 "$R/scripts/probe_affine_pmc.py" $w > "$R/gpurun_out/aff_${w}_kt.log" 2>&1 || { echo "kt $w failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/aff_${w}_sq" -o run -- python3 "$R/scripts/probe_affine_pmc.py" $w > "$R/gpurun_out/aff_${w}_sq.log" 2>&1 || { echo "sq $w failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/aff_${w}_fetch" -o run -- python3 "$R/scripts/probe_affine_pmc.py" $w > "$R/gpurun_out/aff_${w}_fetch.log" 2>&1 || { echo "fetch $w failed"; exit 1; }
done
echo pmc done
