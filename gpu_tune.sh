# Interleaved sweep of the minimum chunk count (tools/tune.py) at 10M and 1M.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/tune19
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
C="MQ_CHUNK_MIN=4; MQ_CHUNK_MIN=1; MQ_CHUNK_MIN=2; MQ_CHUNK_MIN=8"
timeout -k 10 300 python tools/tune.py --subs 1000000 --steps 20 --repeat 2 --configs "$C" > $D/sweep1m.jsonl 2> $D/sweep1m.err || exit 1
timeout -k 10 500 python tools/tune.py --subs 10000000 --steps 10 --repeat 2 --configs "$C" > $D/sweep.jsonl 2> $D/sweep.err || exit 1
