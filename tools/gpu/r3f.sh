# Round 3: merge-set work distribution (MQ_PROF_WORK per-set records) and the walk on a
# byte-sorted batch (a locality experiment for a device-side topic sort).
set -o pipefail
D=gpurun_out/${1:-r3f}
mkdir -p $D
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=8" --work > $D/work_10m.jsonl 2> $D/work_10m.err || { echo "work rc=$?"; tail -5 $D/work_10m.err; exit 1; }
cut -c1-900 $D/work_10m.jsonl
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=8" --sort > $D/sorted_10m.jsonl 2> $D/sorted_10m.err || { echo "sorted rc=$?"; tail -5 $D/sorted_10m.err; exit 1; }
cut -c1-400 $D/sorted_10m.jsonl
