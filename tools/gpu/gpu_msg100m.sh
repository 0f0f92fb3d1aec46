# Config 5 at full scale: 100M retained topics (+1k $SYS) x 100k wildcard filters, Messages path.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/msg100m
mkdir -p $D
timeout -k 10 1000 python bench_messages.py --retained 100000000 --steps 5 --warmup 1 --no-cpu > $D/bench_messages_100m.json 2> $D/bench_messages_100m.err || exit 1
