# Round 5: k_set's record-keyed fold with a 640-slot table (480 visits) against k_merge's 448
# (MQ_OPT_SET_EXP bit 14) — set-pass parity tests, A/B at 1M and 16k topics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/bigtab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "set_pass or spans or merging or pair_hits or partner_map or long_lists or workload_digest" > $O/pytest_set.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=16384 --rounds 3 --check 20000 > $O/ab_1m.json 2> $O/ab_1m.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --topics 16384 --steps 100 --variants 18=0 18=16384 --rounds 3 --check 16384 > $O/ab_16k.json 2> $O/ab_16k.err || exit 1
