# Round 5 validation: the whole GPU suite, smoke(), the default bench line, the 16k-topic batch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit $?
