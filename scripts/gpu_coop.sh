set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_large_parity.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r2c_tests.log; exit 1; }
tail -3 gpurun_out/r2c_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/r2c_bench_coop.json 2> gpurun_out/r2c_bench_coop.err || { echo "bench failed"; tail -20 gpurun_out/r2c_bench_coop.err; exit 1; }
MC_COOPERATIVE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/r2c_bench_plain.json 2> gpurun_out/r2c_bench_plain.err || { echo "bench plain failed"; tail -20 gpurun_out/r2c_bench_plain.err; exit 1; }
python -c "
import json
for f in ['coop','plain']:
    d=json.load(open('gpurun_out/r2c_bench_%s.json'%f)); print(f, d['value']/1e6, d['roofline']['launch_ms'], d['ms_per_step'])
"
