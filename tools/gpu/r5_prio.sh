# Round 5: heavy merge sets at issue priority 3 (MQ_OPT_SET_EXP bit 15) A/B at 16k and 1M topics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/prio
mkdir -p $O
timeout -k 10 300 python -u tools/ab_options.py --topics 16384 --steps 100 --variants 18=0 18=32768 --rounds 3 --check 16384 > $O/ab_16k.json 2> $O/ab_16k.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=32768 --rounds 3 --check 20000 > $O/ab_1m.json 2> $O/ab_1m.err || exit 1
timeout -k 10 300 python -u tests/../tools/ab_options.py --subs 1000000 --variants 18=0 18=32768 --rounds 3 --check 20000 > $O/ab_c2.json 2> $O/ab_c2.err || exit 1
