# Round 5 validation: the whole GPU suite, smoke(), the default bench line, the 16k-topic batch, 8 shards
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/full2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit $?
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit $?
