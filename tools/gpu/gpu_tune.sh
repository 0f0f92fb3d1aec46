# Interleaved sweep of the minimum chunk count (tools/tune.py) at 10M and 1M.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/tune21
mkdir -p $D
true
C="MQ_SUBBATCH_TOPICS=4194304; MQ_SUBBATCH_TOPICS=524288; MQ_SUBBATCH_TOPICS=262144; MQ_SUBBATCH_TOPICS=524288 MQ_CHUNK_TAIL=8"
timeout -k 10 300 python tools/tune.py --subs 1000000 --steps 20 --repeat 2 --configs "$C" > $D/sweep1m.jsonl 2> $D/sweep1m.err || exit 1
timeout -k 10 500 python tools/tune.py --subs 10000000 --steps 10 --repeat 2 --configs "$C" > $D/sweep.jsonl 2> $D/sweep.err || exit 1
