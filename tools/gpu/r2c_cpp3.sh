# The C++ host mirror test with per-test progress (which test does not return).
D=gpurun_out/${1:-r2c_cpp3}
mkdir -p $D
( time timeout -k 5 100 ./mqtt-server_amd/build/test_topics_index ) > $D/cpp.log 2>&1; echo "cpp rc=$?"; cat $D/cpp.log
