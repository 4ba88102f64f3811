#!/bin/bash
# Extra GPU tests, then the config-5 NUTS bench line (with its CPU baseline)
# and a rocprofv3 kernel trace of the same workload.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-np}
TESTS=${2:-tests/test_gpu_kernel_note.py}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 400 python -u -m pytest $TESTS -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --workload nuts > gpurun_out/${TAG}_nuts_bench.json 2> gpurun_out/${TAG}_nuts_bench.err || { echo "nuts bench failed"; tail -5 gpurun_out/${TAG}_nuts_bench.err; exit 1; }
cat gpurun_out/${TAG}_nuts_bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_nuts_kt" -o run -- python3 "$R/bench.py" --workload nuts --no-cpu-baseline > "$R/gpurun_out/${TAG}_nuts_kt.log" 2>&1 || { echo "nuts kt failed"; exit 1; }
echo done
