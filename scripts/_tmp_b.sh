set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 100 --warmup 30 --no-cpu-baseline > gpurun_out/bsl1.json 2> gpurun_out/bsl1.err || { tail -20 gpurun_out/bsl1.err; exit 1; }
cat gpurun_out/bsl1.json
