# GPU parity suite only.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t/pytest_gpu.log 2>&1
