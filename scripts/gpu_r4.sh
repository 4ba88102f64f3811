#!/bin/bash
# Round-4 GPU pass on one box: selected GPU tests (args after the tag; "all"
# = the whole -m gpu suite, "none" = skip), then optional steps picked by
# environment flags: BENCH=1 the default bench line, DF=1 the driver's flags,
# EXPR=1 the expression-throughput probe, SMOKE=1 smoke().  Every GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r4}
shift
SEL="$@"
if [ "$SEL" != "none" ]; then
  if [ "$SEL" = "all" ] || [ -z "$SEL" ]; then SEL="tests -m gpu"; fi
  timeout -k 10 900 python -u -m pytest $SEL -v -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.log | head -40; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_gpu_tests.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ -n "$EXPR" ]; then
  timeout -k 10 300 python -u scripts/bench_expr.py > gpurun_out/${TAG}_bench_expr.log 2>&1 || { echo "bench_expr failed"; tail -5 gpurun_out/${TAG}_bench_expr.log; exit 1; }
  tail -6 gpurun_out/${TAG}_bench_expr.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('bench', d['value']/1e6, d['roofline']['frac'], d['roofline']['launch_ms'])"
fi
if [ -n "$DF" ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver_flags.json 2> gpurun_out/${TAG}_bench_df.err || { echo "bench df failed"; tail -20 gpurun_out/${TAG}_bench_df.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_driver_flags.json'));print('bench df', d['value']/1e6, d['roofline']['frac'])"
fi
exit 0
