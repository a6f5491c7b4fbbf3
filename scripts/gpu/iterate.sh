#!/bin/bash
# Iteration: parity subset, C2 phase stamps (timing build), lean C2 / C3 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
XFLAG= bash scripts/gpu/tests.sh "parity or fullsize or sharded" iterate | tail -3 || exit 1
GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --config c2 --steps 30 \
  > gpurun_out/phases_c2.txt 2> gpurun_out/phases_c2.err || { tail -20 gpurun_out/phases_c2.err; exit 1; }
cat gpurun_out/phases_c2.txt
bash scripts/gpu/ab.sh c2 GTR_X=0 && bash scripts/gpu/ab.sh c3 GTR_X=0
