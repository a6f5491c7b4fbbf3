#!/bin/bash
# kbench (per-launch times) of several library builds: scripts/gpu/kb_libs.sh "cfg B" build/a build/b ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CB=$1; shift
O=gpurun_out/kb_libs.log
: > $O
for b in "$@"; do
  echo "== $b $CB" >> $O
  GTR_LIB=$PWD/gat-recommendation_amd/$b/libgtr_hip.so timeout -k 10 200 python3 -u scripts/dbg/kbench.py $CB >> $O 2>&1 || { tail -5 $O; exit 1; }
done
grep -v "^/opt\|Warn\|warn" $O
