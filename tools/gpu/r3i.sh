# Round 3: the batching stage's dispatcher phases, 64 and 16 submitters (tools/latency.cpp).
set -o pipefail
D=gpurun_out/${1:-r3i}
mkdir -p $D
for W in 64 16; do
timeout -k 10 300 mqtt-server_amd/build/latency 10000000 2 $W > $D/latency_10m_w$W.jsonl 2> $D/latency_10m_w$W.err || { echo "latency rc=$?"; tail -5 $D/latency_10m_w$W.err; exit 1; }
grep Batcher $D/latency_10m_w$W.jsonl
done
