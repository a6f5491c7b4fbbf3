#!/bin/bash
# Phase stamps of the split path's row kernels (timing build). usage: phases.sh "CFG:B ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for cb in ${1:-c3:1024}; do
  GTR_SPLIT=1 GTR_LIB=$PWD/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 200 \
    python3 -u scripts/split_phases.py ${cb%%:*} ${cb##*:} 2>&1 | grep -v "amdgpu.ids" || exit 1
done
