#!/bin/bash
# A/B of the step tail: parity subset on the new library, then the lean bench on the base
# build (GTR_LIB=build/base) and the new one at C2, C3 B=8192, C5 B=1024, C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
XFLAG= bash scripts/gpu/tests.sh "${1:-lazy or lagged or fused_steps or sharded or dp}" abtail
rc=$?; [ $rc -le 1 ] || exit $rc
B=$PWD/gat-recommendation_amd/build/base/libgtr_hip.so
N=$PWD/gat-recommendation_amd/build/libgtr_hip.so
AB_EXTRA="" bash scripts/gpu/ab.sh c2 "GTR_LIB=$B" "GTR_LIB=$N" || exit 1
AB_EXTRA="--batch-size 8192" bash scripts/gpu/ab.sh c3 "GTR_LIB=$B" "GTR_LIB=$N" || exit 1
AB_EXTRA="--batch-size 1024" bash scripts/gpu/ab.sh c5 "GTR_LIB=$B" "GTR_LIB=$N" || exit 1
AB_EXTRA="" bash scripts/gpu/ab.sh c5 "GTR_LIB=$B" "GTR_LIB=$N" || exit 1
exit $rc
