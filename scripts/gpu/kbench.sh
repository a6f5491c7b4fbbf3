#!/bin/bash
# Per-kernel timing variants (scripts/dbg/kbench.py) of the large-batch layer paths.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/kbench_${1:-x}.log
: > $O
run() { echo "== $*" >> $O; env "$@" timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${CFG:-c3} ${BB:-8192} >> $O 2>&1 || { tail -5 $O; exit 1; }; }
run GTR_SPLIT=1
run GTR_SPLIT=1 GTR_ATTN=group
run GTR_SPLIT=0
[ -f gat-recommendation_amd/build/probe/libgtr_hip.so ] && run GTR_SPLIT=1 GTR_LIB=$PWD/gat-recommendation_amd/build/probe/libgtr_hip.so
run GTR_SPLIT=1 GTR_GEMM_GRID=128
CFG=c5 BB=1024 run GTR_SPLIT=1
CFG=c5 BB=1024 run GTR_SPLIT=0
grep -v "^/opt\|Warn\|warn" $O
