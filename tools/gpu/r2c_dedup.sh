# Merge-set dedup on the GPU: parity with dedup on, 10M/1M span step with dedup on vs off,
# the 10M headline parity test with dedup on, and a bench line with dedup on.
set -o pipefail
D=gpurun_out/${1:-r2c_dedup}
mkdir -p $D
MQ_ENGINE_OPTIONS=12=1 bash tools/gpu/r2b_tune.sh ${1:-r2c_dedup} "12=1;12=0" || exit 1
MQ_ENGINE_OPTIONS=12=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 400 --timeout-method thread > $D/scale.log 2>&1 || { echo "scale rc=$?"; tail -20 $D/scale.log; exit 1; }
tail -1 $D/scale.log
MQ_ENGINE_OPTIONS=12=1 timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > $D/bench_dd.json 2> $D/bench_dd.err || { echo "bench rc=$?"; exit 1; }
python tools/show.py $D/bench_dd.json
