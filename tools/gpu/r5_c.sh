# Round 5: the set pass's big-gather fold A/B (MQ_OPT_SET_EXP: 0 one pass, 1024 two passes, 2048 any,
# 512 partner links) at 10M subscriptions, after its parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread \
  -k "set_pass or many_merging or many_pair_hits or long_lists" > $O/pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 0 512 1024; do
  MQ_ENGINE_OPTIONS=18=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_exp$v.json 2> $O/bench_exp$v.err || exit 1
done
exit $rc
