#!/bin/bash
# One-slice lane-resident kernel: sliced tests, the headline bench, configs 2 and 5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-lr1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliced.py -v -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -50
if [ $rc -ne 0 ]; then grep -B5 -A30 "Error\|assert" gpurun_out/${TAG}_tests.log | head -80; exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 100 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));r=d['roofline'];print(d['value']/1e6,'M steps/s', r['kernel_ms'],'ms', r['frac'])"
timeout -k 10 300 python scripts/bench_configs.py > gpurun_out/${TAG}_configs.json 2> gpurun_out/${TAG}_configs.err || { echo "configs failed"; tail -30 gpurun_out/${TAG}_configs.err; exit 1; }
cat gpurun_out/${TAG}_configs.json
