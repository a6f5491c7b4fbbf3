#!/bin/bash
# Column-sliced tail windows: full GPU suite, then per-launch timing with and without
# (GTR_TAIL_COLS=0) at C3 B=8192 and C4 B=1024.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_tailcols.log 2>&1 || { tail -40 gpurun_out/t_tailcols.log; exit 1; }
tail -3 gpurun_out/t_tailcols.log
fi
for v in GTR_TAIL_COLS=1 GTR_TAIL_COLS=0 GTR_TAIL_COLS=1; do
  for cb in ${CBS:-c3:8192 c5:8192}; do
    echo "== $v $cb"
    env $v GTR_SPLIT=1 timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${cb%%:*} ${cb##*:} 2>&1 | grep "^{" || exit 1
  done
done
