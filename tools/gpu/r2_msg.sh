# GPU suite, the Messages bench (level-order image vs particle walk, 10M retained), the
# update-path bench. Each step under its own time limit; stop at the first failure.
set -o pipefail
D=gpurun_out/${1:-r2_msg}
mkdir -p $D
bash tools/gpu/r2_suite.sh ${1:-r2_msg} || exit 1
timeout -k 10 400 python -u bench_messages.py --retained 10000000 > $D/msg_img.json 2> $D/msg_img.err || { echo "msg img rc=$?"; tail -5 $D/msg_img.err; exit 1; }
cat $D/msg_img.json
timeout -k 10 300 python -u bench_messages.py --retained 10000000 --walk --no-cpu > $D/msg_walk.json 2> $D/msg_walk.err || { echo "msg walk rc=$?"; tail -5 $D/msg_walk.err; exit 1; }
cat $D/msg_walk.json
timeout -k 10 400 python -u tools/bench_update.py --subs 10000000 --retained 10000000 > $D/update.json 2> $D/update.err || { echo "update rc=$?"; tail -5 $D/update.err; exit 1; }
cat $D/update.json
