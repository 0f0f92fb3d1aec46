# Round 3 final evidence (secondary): Messages at 10M retained (bench line, PMC passes), config 5
# at full size (100M retained, oracle side from profiles/r02/msg100m_oracle.json: same seeds and
# sizes), config 4 (50M IoT subscriptions).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3v}
mkdir -p $D
timeout -k 10 400 python -u bench_messages.py --retained 10000000 > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -5 $D/msg_10m.err; exit 1; }
cut -c1-400 $D/msg_10m.json
cd /tmp && export TMPDIR=/tmp
KR="k_msgq|k_msg_copy"
MARGS="--retained 10000000 --configs 19=1 --repeat 1 --steps 3"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/mfetch -o run -- python3 $R/tools/tune_msg.py $MARGS > $D/mfetch.json 2> $D/mfetch.err || { echo "mfetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/mwrite -o run -- python3 $R/tools/tune_msg.py $MARGS > $D/mwrite.json 2> $D/mwrite.err || { echo "mwrite rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/mfetch $D/mwrite --pmc > $D/msg_pmc.json
grep -B2 -A7 hbm_bytes $D/msg_pmc.json | head -60
timeout -k 10 600 python -u bench_messages.py --retained 100000000 --oracle-file profiles/r02/msg100m_oracle.json > $D/msg_100m.json 2> $D/msg_100m.err || { echo "msg100m rc=$?"; tail -5 $D/msg_100m.err; exit 1; }
cut -c1-400 $D/msg_100m.json
timeout -k 10 400 python -u bench.py --mix iot --subs 50000000 --no-cpu > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -5 $D/bench_iot_50m.err; exit 1; }
cut -c1-400 $D/bench_iot_50m.json
