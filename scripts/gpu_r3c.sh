#!/bin/bash
# Round-3 (session 2) GPU pass: the whole GPU suite, smoke(), the default
# bench line and the driver's flags.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-v28}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.log | head -40; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('bench', d['value']/1e6, d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver_flags.json 2> gpurun_out/${TAG}_bench_df.err || { echo "bench df failed"; tail -20 gpurun_out/${TAG}_bench_df.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_driver_flags.json'));print('bench df', d['value']/1e6, d['roofline']['frac'])"
