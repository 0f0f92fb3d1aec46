# Parity, then interleaved knob sweep (tools/tune.py) at 1M and 10M.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/tune13
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
C="MQ_COPY_BLOCKS_PER_CU=8; MQ_COPY_BLOCKS_PER_CU=0; MQ_SERIAL=1"
timeout -k 10 300 python tools/tune.py --subs 1000000 --steps 20 --repeat 2 --configs "$C" > $D/sweep1m.jsonl 2> $D/sweep1m.err || exit 1
timeout -k 10 500 python tools/tune.py --subs 10000000 --steps 10 --repeat 2 --configs "$C" > $D/sweep.jsonl 2> $D/sweep.err || exit 1
