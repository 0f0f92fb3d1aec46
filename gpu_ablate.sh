set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for a in 0 2 8 16 24 32 64 96 120; do
  MQ_EMIT_ABLATE=$a timeout -k 10 200 python bench.py --subs 1000000 --steps 3 --warmup 1 --no-cpu > gpurun_out/abl/a$a.json 2> gpurun_out/abl/a$a.err || exit 1
done
