# Final tree with the edge table at load <= 1/4: smoke, full GPU suite, load 1/8 probe, then
# rocprofv3 trace + PMC passes and the default bench line (r2c_final.sh, without Messages).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r2c_end2}
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
MQ_ENGINE_OPTIONS=13=8 timeout -k 10 300 python -u bench.py --no-cpu --steps 10 > $D/bench_load8.json 2> $D/bench_load8.err || { echo "b8 rc=$?"; tail -5 $D/bench_load8.err; exit 1; }
python tools/show.py $D/bench_load8.json
sed -i 's/^timeout -k 10 500 python -u bench_messages.py.*$/true/; s/^cut -c1-600.*$/true/' tools/gpu/r2c_final.sh
bash tools/gpu/r2c_final.sh ${1:-r2c_end2} || exit 1
