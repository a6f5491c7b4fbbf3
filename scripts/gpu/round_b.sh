#!/bin/bash
# Round-2 artifacts, part B: C3 at B = 8192 and C5 (1M-row table, lazy, B = 8192).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/profile.sh c3 c3_b8192 --batch-size 8192 --num-batches 8 || exit 1
bash scripts/gpu/profile.sh c5 c5 --num-batches 8 || exit 1
