# Paired-slot probing: parity file, then the 10M span step (bench.py --no-cpu).
set -o pipefail
D=gpurun_out/${1:-r2c_pair}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -1 $D/parity.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 > $D/bench.json 2> $D/bench.err || { echo "bench rc=$?"; tail -5 $D/bench.err; exit 1; }
python tools/show.py $D/bench.json
