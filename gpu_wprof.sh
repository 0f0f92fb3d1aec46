set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wprof
for a in 0 8 1; do
  MQ_EMIT_PROF=1 MQ_EMIT_ABLATE=$a timeout -k 10 200 python bench.py --subs 1000000 --steps 2 --warmup 0 --no-cpu > gpurun_out/wprof/a$a.json 2> gpurun_out/wprof/a$a.err || exit 1
done
