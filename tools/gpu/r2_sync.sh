# GPU suite + update-path bench (sync under churn after the 512-byte page / scatter upload)
set -o pipefail
D=gpurun_out/${1:-r2_sync}
mkdir -p $D
bash tools/gpu/r2_suite.sh ${1:-r2_sync} || exit 1
timeout -k 10 600 python -u tools/bench_update.py --subs 10000000 --retained 10000000 > $D/update.json 2> $D/update.err || { echo "update rc=$?"; tail -5 $D/update.err; exit 1; }
cat $D/update.json
