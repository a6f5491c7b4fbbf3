#!/bin/bash
# Full GPU suite, then per-launch timing of the default build at the given configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_suite.log 2>&1 || { tail -40 gpurun_out/t_suite.log; exit 1; }
tail -2 gpurun_out/t_suite.log
for cb in ${CBS:-c4:1024 c5:1024 c3:8192}; do
  echo "== $cb"
  GTR_SPLIT=1 timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${cb%%:*} ${cb##*:} 2>&1 | grep "^{" || exit 1
done
