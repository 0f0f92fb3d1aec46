# Round-end confirmation on a fresh box with the tree as committed: GPU parity suite, smoke(),
# and the driver's default bench invocation.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/confirm
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || exit 1
