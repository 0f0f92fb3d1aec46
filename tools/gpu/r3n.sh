# Round 3 (session 2): attribution of the merge set pass's time (MQ_OPT_SET_EXP 18 bits; results
# of those steps are wrong by design, timing only) at 10M subscriptions.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3n}
mkdir -p $D
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "18=0;18=1;18=2;18=4;18=8;18=15" > $D/setexp_10m.jsonl 2> $D/setexp_10m.err || { echo "tune rc=$?"; tail -5 $D/setexp_10m.err; exit 1; }
cut -c1-420 $D/setexp_10m.jsonl
