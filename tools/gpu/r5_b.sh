# Round 5, first GPU pass: per-thread HIP set-up probe, the round's new parity tests (pipelined
# submit error path, bulk subscribe beside a ticket, image edge-table tiers, walk trials, the set
# pass's bit fold), the C++ mirror, then the default bench line (calibration batches, fold-shape
# work counters) and the set pass A/B (MQ_OPT_SET_EXP bit 9: big gathers through partner links).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/b
mkdir -p $O

timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread \
  -k "pipelined or set_pass or many_merging or many_pair_hits or long_lists or spans_device_digest or cpp_host_mirror" \
  > $O/pytest.log 2>&1
rc=$?
# test failures (1) still measure; anything else (a fault, an abort, a time limit) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
MQ_ENGINE_OPTIONS=18=512 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_links.json 2> $O/bench_links.err || exit 1
exit $rc
