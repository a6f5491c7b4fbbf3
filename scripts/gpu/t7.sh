#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
XFLAG= bash scripts/gpu/tests.sh "" beginfused || exit 1
GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/dbg_phases.py c2 > gpurun_out/ph.txt 2> gpurun_out/ph.err || { tail -5 gpurun_out/ph.err; exit 1; }
cat gpurun_out/ph.txt
