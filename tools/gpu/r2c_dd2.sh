# Merge-set dedup after the wave-leader insert and the representative list: parity with dedup
# on, then the span step with dedup on vs off at 10M and 1M subscriptions.
set -o pipefail
D=gpurun_out/${1:-r2c_dd2}
mkdir -p $D
MQ_ENGINE_OPTIONS=12=1 bash tools/gpu/r2b_tune.sh ${1:-r2c_dd2} "12=1;12=0" || exit 1
