set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_sliced.py -q -x > gpurun_out/slk_tests.log 2>&1
rc=$?
tail -15 gpurun_out/slk_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; exit $rc; fi
for v in full; do
timeout -k 10 300 python scripts/stamps_sliced.py 16 256 $v > gpurun_out/slk_$v.log 2>&1 || { tail -20 gpurun_out/slk_$v.log; exit 1; }
grep -v " 0       0       0" gpurun_out/slk_$v.log
done
