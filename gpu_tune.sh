# Interleaved chunk-size sweep (tools/tune.py) at 10M and 1M.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/tune18
mkdir -p $D
C="MQ_CHUNK_TAIL=8; MQ_CHUNK_TAIL=0; MQ_CHUNK_ROWS=4000000000 MQ_CHUNK_TAIL=8; MQ_CHUNK_ROWS=4000000000 MQ_CHUNK_TAIL=0; MQ_CHUNK_TAIL=16"
timeout -k 10 500 python tools/tune.py --subs 10000000 --steps 10 --repeat 2 --configs "$C" > $D/sweep.jsonl 2> $D/sweep.err || exit 1
true
