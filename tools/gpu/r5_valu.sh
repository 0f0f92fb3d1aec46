set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05/valu
timeout -k 10 60 ./tools/valubench > gpurun_out/r05/valu/valubench.jsonl 2>&1 || exit 1
