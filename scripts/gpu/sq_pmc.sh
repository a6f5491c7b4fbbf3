#!/bin/bash
# SQ wave-state counters (one --pmc pass, 7 SQ counters) of the split-path kernels at one
# config, via scripts/dbg/kbench.py -> gpurun_out/sq_<cfg>/  usage: sq_pmc.sh [cfg] [B]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp GTR_SPLIT=1
CFG=${1:-c3}; B=${2:-8192}
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace \
  -d gpurun_out/sq_${CFG}_${B} -o run --output-format csv -- python3 scripts/dbg/kbench.py $CFG $B 6 \
  > gpurun_out/sq_${CFG}_${B}.log 2>&1
rc=$?
tail -3 gpurun_out/sq_${CFG}_${B}.log
exit $rc
