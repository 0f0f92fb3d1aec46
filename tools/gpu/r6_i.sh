#!/bin/bash
# Round 6: the north star's "hot trie levels staged in LDS", bounded by attribution (development
# library): the walk with its level-0 probes, and with its level-0 and level-1 probes, looked up
# ahead of it by a kernel of their own (MQ_OPT_WALK_EXP bits 0 / 1), in one process, results equal
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/i
mkdir -p $O
MQ_LIB_DIR=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_dev timeout -k 10 400 python -u tools/ab_options.py --check 4096 --variants 24=0 24=1 24=2 --rounds 3 > $O/ab_hint.json 2> $O/ab_hint.err || exit 1
