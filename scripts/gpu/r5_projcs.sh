#!/bin/bash
# Column-sliced k_proj at small batches: split-path parity tests, then per-launch timing
# with GTR_PROJ_CS=1 / 4 (and 2 tiles per stream) at C4 B=1024, C5 B=1024, C3 B=8192.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_ffn.py tests/test_gpu_c4.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_projcs.log 2>&1 || { tail -40 gpurun_out/t_projcs.log; exit 1; }
tail -2 gpurun_out/t_projcs.log
for v in GTR_PROJ_CS=1 GTR_PROJ_CS=4 GTR_PROJ_CS=4,GTR_PROJ_CS_TPB=2 GTR_PROJ_CS=1 GTR_PROJ_CS=4; do
  for cb in ${CBS:-c4:1024 c5:1024}; do
    echo "== $v $cb"
    env ${v//,/ } GTR_SPLIT=1 timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${cb%%:*} ${cb##*:} 2>&1 | grep "^{" || exit 1
  done
done
