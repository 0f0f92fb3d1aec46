# Round 5: set pass big-gather fold A/B in one process (tools/ab_options.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/e
mkdir -p $O
timeout -k 10 500 python -u tools/ab_options.py --variants 18=0 18=512 18=1024 --rounds 4 > $O/ab_set.json 2> $O/ab_set.err || exit 1
