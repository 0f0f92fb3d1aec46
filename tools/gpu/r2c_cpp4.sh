# The reverted tree: the C++ host mirror test through pytest (as the suite runs it), then the
# parity file.
set -o pipefail
D=gpurun_out/${1:-r2c_cpp4}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 170 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -3 $D/parity.log
