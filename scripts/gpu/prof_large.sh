#!/bin/bash
# Kernel stats + PMC traffic of the large-batch single-GPU lines (C3 B = 8192,
# C5 B = 8192 and 1024: the lazy table's one-RMW moments), after a DP / lazy test pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export ROUND=${ROUND:-r04}
bash scripts/gpu/tests.sh "distributed or lazy or dp or c5s" dplazy || exit 1
bash scripts/gpu/profile.sh c3 c3_b8192 --batch-size 8192 || exit 1
bash scripts/gpu/profile.sh c5 c5 || exit 1
bash scripts/gpu/profile.sh c5 c5_b1024 --batch-size 1024 || exit 1
