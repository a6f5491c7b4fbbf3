#!/bin/bash
# Round-3 iteration: parity subset, then C5 B=1024 kernel stats and per-kernel variants.
# usage: scripts/gpu/iter3.sh TAG [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-it}
XFLAG= bash scripts/gpu/tests.sh "${2:-parity or sharded or distributed or split}" ${TAG}
rc=$?; [ $rc -le 1 ] || exit $rc
ROUND=r03 PMC=0 bash scripts/gpu/profile.sh c5 ${TAG}_c5b1024 --batch-size 1024 --c1-reps 0 || exit 1
GTR_RO_WAVE_MIN_B=1024 timeout -k 10 200 python3 -u scripts/dbg/kbench.py c5 1024 > gpurun_out/${TAG}_kb_wave.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/dbg/kbench.py c5 1024 > gpurun_out/${TAG}_kb.log 2>&1 || exit 1
grep "{" gpurun_out/${TAG}_kb_wave.log gpurun_out/${TAG}_kb.log
exit $rc
