# Round 5: k_set with the visit-sized big-fold table vs k_merge's set pass (product library), then
# the fused walk's register budget and group size (development library: 9=1 no wave constraint,
# 15=8 eight-lane groups)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g
mkdir -p $O

MQ_LIB_DIR=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_dev timeout -k 10 300 python -u tools/ab_options.py --check 4096 --variants 15=16 15=16,9=1 15=8 --rounds 3 > $O/ab_walk.json 2> $O/ab_walk.err || exit 1
