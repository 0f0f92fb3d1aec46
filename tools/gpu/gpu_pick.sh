# k_pick parity + its cost inside the 10M step.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/pick
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_select.py -x -v --timeout 120 --timeout-method thread > $D/pytest_select.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu --select-shared > $D/bench_10m_select.json 2> $D/bench_10m_select.err || exit 1
MQ_SERIAL=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu --select-shared > $D/bench_10m_select_serial.json 2> $D/bench_10m_select_serial.err || exit 1
