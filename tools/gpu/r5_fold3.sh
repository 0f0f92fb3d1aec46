# Round 5: the hash fold's fill, in-process A/B at 1M and 16k topics: 2/3 (default) vs 3/5
# (MQ_OPT_SET_EXP bit 17) vs 3/4 (bit 16), results compared across variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/fold3
mkdir -p $O
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=131072 18=65536 --rounds 3 --check 20000 > $O/ab_1m.json 2> $O/ab_1m.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --topics 16384 --steps 100 --variants 18=0 18=131072 18=65536 --rounds 3 --check 16384 > $O/ab_16k.json 2> $O/ab_16k.err || exit 1
