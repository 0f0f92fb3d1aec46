#!/bin/bash
# round 4 end: smoke and the whole GPU suite on the final tree, then the Messages PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r4end; mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/pytest.log 2>&1; echo "pytest rc=$?"
tail -2 $D/pytest.log
bash $R/tools/gpu/r4mp.sh
