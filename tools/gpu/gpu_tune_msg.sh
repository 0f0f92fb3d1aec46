# k_msg occupancy variants A/B on one box (10M and 1M retained).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/tunemsg
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k messages -x -q --timeout 120 --timeout-method thread > $D/pytest_msg.log 2>&1 || exit 1
timeout -k 10 400 python tools/tune_msg.py --retained 10000000 --configs "1;6;8" --repeat 2 > $D/tune_10m.txt 2> $D/tune_10m.err || exit 1
timeout -k 10 300 python tools/tune_msg.py --retained 1000000 --configs "1;6;8" --repeat 2 > $D/tune_1m.txt 2> $D/tune_1m.err || exit 1
