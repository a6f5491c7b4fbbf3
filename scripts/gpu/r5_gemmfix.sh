#!/bin/bash
# GEMM / weight-gradient pipelines with counted waits: the split-path parity tests, then
# per-launch timing (scripts/dbg/kbench.py) at C3 B=8192 and C4 B=1024.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_split.py tests/test_gpu_ffn.py tests/test_gpu_parity.py} -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gemmfix.log 2>&1 || { tail -40 gpurun_out/t_gemmfix.log; exit 1; }
tail -3 gpurun_out/t_gemmfix.log
for cb in ${CBS:-c3:8192 c4:1024}; do
  echo "== $cb"
  GTR_SPLIT=1 timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${cb%%:*} ${cb##*:} 2>&1 | grep "^{" || exit 1
done
