#!/bin/bash
# round 4: which of bench.py's differences serialises the pipelined submit behind the last copy
set -o pipefail
D=gpurun_out/r4q; mkdir -p $D
for v in "--seq-first" "--torch" "--torch --seq-first"; do
  timeout -k 10 200 python -u tools/e2e_pipe.py 10000000 --expected $v >> $D/e2e_pipe.txt 2>&1 || { echo "e2e $v rc=$?"; tail -5 $D/e2e_pipe.txt; exit 1; }
done
cut -c1-700 $D/e2e_pipe.txt
