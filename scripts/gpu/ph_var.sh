#!/bin/bash
# Phase stamps (C2) of timing-build variants: scripts/gpu/ph_var.sh build/t_A build/t_B ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for B in "$@"; do
  GTR_LIB=gat-recommendation_amd/$B/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --config ${CFG:-c2} --steps 30 > gpurun_out/phv.txt 2> gpurun_out/phv.err || { tail -20 gpurun_out/phv.err; exit 1; }
  echo "== $B"; grep bwd gpurun_out/phv.txt
done
