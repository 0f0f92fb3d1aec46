# Round 5: the 16k-topic batch's kernel timeline (gaps between launches) and the default line
# with the locate_run set pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/k16
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --topics 16384 --steps 50 --warmup 10 --no-cpu > $O/bench_16k_traced.json 2> $O/bench_16k_traced.err || exit 1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "set_pass or spans or merging or pair_hits or partner_map or long_lists or workload_digest" > $O/pytest_set.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
