# Round 3 (session 2): where the Messages count pass spends its time at 10M retained (per-filter
# clocks, fan-out lookups, filters whose frontier outgrew LDS).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3p}
mkdir -p $D
timeout -k 10 400 python -u tools/tune_msg.py --retained 10000000 --configs "8=1" --repeat 1 --work > $D/msgwork_10m.jsonl 2> $D/msgwork_10m.err || { echo "tune rc=$?"; tail -5 $D/msgwork_10m.err; exit 1; }
cat $D/msgwork_10m.jsonl
