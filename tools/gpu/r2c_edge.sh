# Edge table at load <= 1/4 (MQ_OPT_EDGE_LOAD 4) against the default 1/2: parity file with the
# sparse table, then the 10M span step both ways (bench.py --no-cpu).
set -o pipefail
D=gpurun_out/${1:-r2c_edge}
mkdir -p $D
MQ_ENGINE_OPTIONS=13=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -1 $D/parity.log
MQ_ENGINE_OPTIONS=13=4 timeout -k 10 300 python -u bench.py --no-cpu --steps 10 > $D/bench_load4.json 2> $D/bench_load4.err || { echo "b4 rc=$?"; tail -5 $D/bench_load4.err; exit 1; }
python tools/show.py $D/bench_load4.json
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 > $D/bench_load2.json 2> $D/bench_load2.err || { echo "b2 rc=$?"; tail -5 $D/bench_load2.err; exit 1; }
python tools/show.py $D/bench_load2.json
grep -o "edge_capacity': [0-9]*" $D/bench_load4.err $D/bench_load2.err
