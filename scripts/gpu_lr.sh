#!/bin/bash
# Lane-resident kernel session: sliced tests, then a short bench of each kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-lr}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliced.py -v -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -40
if [ $rc -ne 0 ]; then grep -B5 -A30 "Error\|assert" gpurun_out/${TAG}_tests.log | head -80; exit $rc; fi
for k in lanes interpreter; do
timeout -k 10 300 python bench.py --steps 100 --warmup 50 --no-cpu-baseline --slice-kernel $k > gpurun_out/${TAG}_bench_$k.json 2> gpurun_out/${TAG}_bench_$k.err || { echo "bench $k failed"; tail -30 gpurun_out/${TAG}_bench_$k.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$k.json'));r=d['roofline'];print('$k', d['value']/1e6,'M steps/s', r['kernel_ms'],'ms', r['frac'], d['accept_rate'], d['step_size'], d.get('rhat'))"
done
