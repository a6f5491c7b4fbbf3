#!/bin/bash
# Per-kernel timing (scripts/dbg/kbench.py) of the layer paths: fused row groups
# (GTR_SPLIT=0) against the split path (GTR_SPLIT=1) at several batch sizes.
# usage: kbench.sh TAG "CFG:B ..." ["ENV=... ENV=..."]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/kbench_${1:-x}.log
: > $O
run() { echo "== $*" >> $O; env "$@" timeout -k 10 200 python3 -u scripts/dbg/kbench.py $CB >> $O 2>&1 || { tail -5 $O; exit 1; }; }
for cb in ${2:-c3:1024}; do
  CB="${cb%%:*} ${cb##*:}"
  for v in ${3:-GTR_SPLIT=1}; do run ${v//,/ }; done
done
grep -v "^/opt\|Warn\|warn" $O
