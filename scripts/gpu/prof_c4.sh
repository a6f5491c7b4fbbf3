#!/bin/bash
# Kernel stats + PMC traffic of the sharded C4 step at world 1 -- per-rank B = 1024
# on the split layer path (as at N = 8 under SyncBN) and B = 8192.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export ROUND=${ROUND:-r04}
GTR_SPLIT=1 bash scripts/gpu/profile.sh c4 c4_b1024 --global-batch 1024 || exit 1
bash scripts/gpu/profile.sh c4 c4_b8192 --global-batch 8192 || exit 1
