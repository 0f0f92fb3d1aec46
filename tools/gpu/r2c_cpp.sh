# The C++ host mirror test alone (timed), then the parity file, on the reverted tree.
set -o pipefail
D=gpurun_out/${1:-r2c_cpp}
mkdir -p $D
( time timeout -k 5 150 ./mqtt-server_amd/build/test_topics_index ) > $D/cpp.log 2>&1; echo "cpp rc=$?"; tail -5 $D/cpp.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -1 $D/parity.log
