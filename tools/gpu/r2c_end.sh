# End-of-session evidence on the final tree: smoke(), the full GPU suite, then rocprofv3 kernel
# trace + PMC passes of the default step, the default bench line and Messages 10M.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r2c_end}
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
bash tools/gpu/r2c_final.sh ${1:-r2c_end} || exit 1
