# Kernel timeline of the 10M step (rocprofv3 kernel trace, CSV), the config-1 line (10k subs)
# and a 10M step with the device share pick.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/tl
mkdir -p $D
timeout -k 10 300 python bench.py --subs 10000 --clients 1000 --steps 20 --warmup 2 --cpu-seconds 10 > $D/bench_10k.json 2> $D/bench_10k.err || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu --select-shared > $D/bench_10m_select.json 2> $D/bench_10m_select.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $D/trace.log 2>&1 || exit 1
