# Round 5: k_set (the lean set pass) against k_merge's set pass, in one process, after parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/f
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread \
  -k "set_pass or many_merging or many_pair_hits or long_lists or spans_device_digest or host_spans_own or pipelined or workload_digest" > $O/pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=8192 18=512 --rounds 4 > $O/ab_prod.json 2> $O/ab_prod.err || exit 1
timeout -k 10 300 python -u tools/concurrency.py --handles 2 > $O/concurrency.json 2> $O/concurrency.err || exit 1
exit $rc
