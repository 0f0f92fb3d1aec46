# Parity file, then config 5 at full size (GPU side) and config 4 (IoT 50M).
set -o pipefail
D=gpurun_out/${1:-r2c_big2}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -1 $D/parity.log
bash tools/gpu/r2c_msg100.sh ${1:-r2c_big2} || exit 1
bash tools/gpu/r2c_iot.sh ${1:-r2c_big2} || exit 1
