# Round artefacts: parity suite, 10M + 1M bench lines (CPU baseline), kernel-trace stats and
# HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs) of the 10M bench step.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/final4
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 10 --warmup 2 --cpu-seconds 10 > $D/bench_10m.json 2> $D/bench_10m.err || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 20 --warmup 2 --cpu-seconds 10 > $D/bench_1m.json 2> $D/bench_1m.err || exit 1
timeout -k 10 600 python bench.py --topics 10000000 --steps 2 --warmup 1 --no-cpu > $D/bench_10m_10mtopics.json 2> $D/bench_10m_10mtopics.err || exit 1
timeout -k 10 300 python bench.py --subs 10000 --clients 1000 --steps 20 --warmup 2 --cpu-seconds 10 > $D/bench_10k.json 2> $D/bench_10k.err || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu --select-shared > $D/bench_10m_select.json 2> $D/bench_10m_select.err || exit 1
timeout -k 10 600 python bench_messages.py --retained 10000000 --filters 100000 > $D/msg_10m.json 2> $D/msg_10m.err || exit 1
timeout -k 10 300 python bench_messages.py --retained 1000000 --filters 100000 > $D/msg_1m.json 2> $D/msg_1m.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $D/trace.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu > $D/fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $D/write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu > $D/write.log 2>&1 || exit 1
