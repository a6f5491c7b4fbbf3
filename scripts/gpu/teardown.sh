#!/bin/bash
# RCCL teardown probe (MODES="nocapture del reset keep" adds the known hang, last).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in ${MODES:-nocapture del reset}; do
  echo "== $m"
  timeout -k 5 90 python -u scripts/dbg/teardown_probe.py $m 2>&1 | grep -v '^\s*$' | tail -5
  rc=$?
  echo "rc $rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
