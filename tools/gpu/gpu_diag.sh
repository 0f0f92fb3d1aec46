# Diagnosis: share of output rows in big lists (k_desc counters).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/diag2
mkdir -p $D
MQ_MERGE_STATS= timeout -k 10 300 python bench.py --subs 1000000 --steps 1 --warmup 0 --no-cpu > $D/s1m.json 2> $D/s1m.err || exit 1
MQ_MERGE_STATS= timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu > $D/s10m.json 2> $D/s10m.err || exit 1
