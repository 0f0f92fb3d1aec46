# GPU test suite only (-m gpu), log to gpurun_out/<name>/pytest_gpu.log
set -o pipefail
D=gpurun_out/${1:-r2_suite}
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $D/pytest_gpu.log
grep -E "passed|failed|PASSED|FAILED" $D/pytest_gpu.log | tail -5
grep -E "test_headline|test_iot_5m|test_two_rank" $D/pytest_gpu.log
exit $rc
