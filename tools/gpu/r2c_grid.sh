# Merge set pass: persistent waves (14=0) against a wavefront per set (14=1), 10M and 1M; parity
# file with 14=1 first.
set -o pipefail
D=gpurun_out/${1:-r2c_grid}
mkdir -p $D
MQ_ENGINE_OPTIONS=14=1 bash tools/gpu/r2b_tune.sh ${1:-r2c_grid} "14=0;14=1" || exit 1
