# Round 3 (session 2): Messages export threshold sweep at 10M retained (MQ_OPT_MSG_EXPORT 19).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3r}
mkdir -p $D
timeout -k 10 400 python -u tools/tune_msg.py --retained 10000000 --configs "19=2048;19=1024;19=512;19=256;19=128" --repeat 2 --work > $D/msgthr_10m.jsonl 2> $D/msgthr_10m.err || { echo "tune rc=$?"; tail -5 $D/msgthr_10m.err; exit 1; }
cut -c1-700 $D/msgthr_10m.jsonl
