#!/bin/bash
# Round-3 profiles: kernel stats (+ PMC for C2) of the default C2 line, C3 at B = 8192,
# C5 at B = 8192 and B = 1024 (the strong-scaling per-rank batch at N = 8).
# usage: scripts/gpu/prof3.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-p}
ROUND=r03 PMC=${PMC_C2:-1} bash scripts/gpu/profile.sh c2 ${T}_c2 --c1-reps 0 || exit 1
ROUND=r03 PMC=${PMC_BIG:-0} bash scripts/gpu/profile.sh c3 ${T}_c3_b8192 --batch-size 8192 --c1-reps 0 || exit 1
ROUND=r03 PMC=${PMC_BIG:-0} bash scripts/gpu/profile.sh c5 ${T}_c5 --c1-reps 0 || exit 1
ROUND=r03 PMC=${PMC_BIG:-0} bash scripts/gpu/profile.sh c5 ${T}_c5_b1024 --batch-size 1024 --c1-reps 0 || exit 1
