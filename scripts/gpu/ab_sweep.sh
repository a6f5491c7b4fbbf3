#!/bin/bash
# A/B of the sweep slices' zero-gradient update inside the layer kernels (apply vs
# apply_zero): lean bench of the base build (GTR_LIB=build/base) and the tree's at C2 / C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=$PWD/gat-recommendation_amd/build/base/libgtr_hip.so
N=$PWD/gat-recommendation_amd/build/libgtr_hip.so
bash scripts/gpu/ab.sh c3 "GTR_LIB=$B" "GTR_LIB=$N" || exit 1
bash scripts/gpu/ab.sh c2 "GTR_LIB=$B" "GTR_LIB=$N" || exit 1
