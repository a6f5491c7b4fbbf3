#!/bin/bash
# round 5: split-path attention kernels -- parity subset, then per-launch timings (old vs new)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${TESTK:-split or edge_cases or long_sessions or c4}" > gpurun_out/t_attn.log 2>&1 || { tail -60 gpurun_out/t_attn.log; exit 1; }
tail -3 gpurun_out/t_attn.log
bash scripts/gpu/kbench.sh attn "${KB:-c3:8192 c4:1024}" "GTR_SPLIT=1,GTR_ATTN=rows GTR_SPLIT=1" || exit 1
