# Round 5: the whole GPU suite on k_msgq / k_walk reading their arguments at their uses and k_set's
# 640-slot record-keyed fold; A/B of that table against k_merge's 448 (MQ_OPT_SET_EXP bit 14) at 1M
# and 16k topics; Messages at 10M retained; the default line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/combo
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=16384 --rounds 3 --check 20000 > $O/ab_1m.json 2> $O/ab_1m.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --topics 16384 --steps 100 --variants 18=0 18=16384 --rounds 3 --check 16384 > $O/ab_16k.json 2> $O/ab_16k.err || exit 1
timeout -k 10 400 python -u bench_messages.py > $O/msg_10m.json 2> $O/msg_10m.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
