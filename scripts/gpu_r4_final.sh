#!/bin/bash
# Round-4 final pass on one box: the whole GPU suite and smoke(), the default
# bench line, the driver's flags, the small / medium shape lines and the NUTS
# lines (config 5 and the Large shape).  Every GPU step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-v41}
SMOKE=1 BENCH=1 DF=1 bash scripts/gpu_r4.sh $TAG all || exit 1
for sh in small medium; do
  timeout -k 10 300 python -u bench.py --shape $sh --no-cpu-baseline > gpurun_out/${TAG}_bench_$sh.json 2> gpurun_out/${TAG}_bench_$sh.err || { echo "bench $sh failed"; tail -20 gpurun_out/${TAG}_bench_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$sh.json'));print('$sh', d['value']/1e6, d['roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --workload nuts > gpurun_out/${TAG}_bench_nuts.json 2> gpurun_out/${TAG}_bench_nuts.err || { echo "bench nuts failed"; tail -20 gpurun_out/${TAG}_bench_nuts.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_nuts.json'));print('nuts', d['value']/1e6, d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --workload nuts --nuts-model hier --shape large --chains 256 --steps 20 --warmup 20 > gpurun_out/${TAG}_bench_nuts_large.json 2> gpurun_out/${TAG}_bench_nuts_large.err || { echo "bench nuts large failed"; tail -20 gpurun_out/${TAG}_bench_nuts_large.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_nuts_large.json'));print('nuts large', d['value']/1e6, d['roofline']['frac'])"
echo final done
