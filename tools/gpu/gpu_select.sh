# Device SelectShared (k_pick) parity, then the full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sel
timeout -k 10 300 python -u -m pytest tests/test_gpu_select.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sel/pytest_select.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sel/pytest_gpu.log 2>&1
