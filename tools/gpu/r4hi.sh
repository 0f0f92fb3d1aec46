# r4i (the fold's parity and A/B), the copy/compute overlap probe, then the C++ mirror tests
# (copy-on-write liveness: slowest update under three readers).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4hi}
mkdir -p $D
bash tools/gpu/r4i.sh ${1:-r4hi} || exit 1
timeout -k 10 300 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -30 $D/cpp.log; exit 1; }
grep -E "slowest|over 2 ms|passed|FAIL|held" $D/cpp.log
