# GPU suite, then the update-path bench (bulk build vs per-entry, churn + mq_sync) at 10M subs
set -o pipefail
D=gpurun_out/${1:-r2_update}
mkdir -p $D
bash tools/gpu/r2_suite.sh ${1:-r2_update} || exit 1
timeout -k 10 600 python -u tools/bench_update.py --subs 10000000 --retained ${2:-10000000} \
  > $D/update.json 2> $D/update.err
rc=$?
echo "bench_update rc=$rc"; cat $D/update.json; tail -3 $D/update.err
exit $rc
