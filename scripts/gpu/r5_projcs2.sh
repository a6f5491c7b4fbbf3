#!/bin/bash
# k_proj column slices: tiles per stream sweep at C4 / C5 B=1024 (per-launch timing).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in ${VARS:-GTR_PROJ_CS=1 GTR_PROJ_CS_TPB=2 GTR_PROJ_CS_TPB=3 GTR_PROJ_CS_TPB=4 GTR_PROJ_CS_TPB=6 GTR_PROJ_CS=1 GTR_PROJ_CS_TPB=3}; do
  for cb in ${CBS:-c4:1024 c5:1024}; do
    echo "== $v $cb"
    env ${v//,/ } GTR_SPLIT=1 timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${cb%%:*} ${cb##*:} 2>&1 | grep "^{" || exit 1
  done
done
