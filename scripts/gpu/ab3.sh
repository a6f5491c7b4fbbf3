#!/bin/bash
# A/B of the large-batch layer kernels: parity subset on the new library, then kbench
# (per-launch times) of the base build (GTR_LIB=build/base) and the new one.
# usage: scripts/gpu/ab3.sh TAG [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
XFLAG= bash scripts/gpu/tests.sh "${2:-split or c4 or large_batch or sharded}" ${TAG}
rc=$?; [ $rc -le 1 ] || exit $rc
O=gpurun_out/${TAG}_kb.log
: > $O
for cfg in "c3 8192" "c5 1024"; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/gat-recommendation_amd/build/base/libgtr_hip.so; else L=$PWD/gat-recommendation_amd/build/libgtr_hip.so; fi
    echo "== $lib $cfg" >> $O
    GTR_LIB=$L timeout -k 10 200 python3 -u scripts/dbg/kbench.py $cfg >> $O 2>&1 || { tail -5 $O; exit 1; }
  done
done
grep -v "^/opt\|Warn\|warn" $O
exit $rc
