# Round 5: which step holds the handle lock when TestConcurrentReadersAndUpdates sees a 15 ms
# match (MQ_SLOW_MS=4 prints the slow calls' milestones), three runs of the C++ test; then the
# rest of the combo: A/B of k_set's fold table, Messages at 10M, the default line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/slow
mkdir -p $O
for k in 1 2 3; do
  MQ_SLOW_MS=4 timeout -k 10 120 ./mqtt-server_amd/build/test_topics_index > $O/cpp$k.out 2> $O/cpp$k.err
  echo "run $k rc=$?" >> $O/cpp_rc.txt
done
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=16384 --rounds 3 --check 20000 > $O/ab_1m.json 2> $O/ab_1m.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --topics 16384 --steps 100 --variants 18=0 18=16384 --rounds 3 --check 16384 > $O/ab_16k.json 2> $O/ab_16k.err || exit 1
timeout -k 10 400 python -u bench_messages.py > $O/msg_10m.json 2> $O/msg_10m.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
