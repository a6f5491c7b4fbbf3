#!/bin/bash
# Kernel stats + PMC traffic of C2 (then the full default bench line, as the
# driver runs it) and C3 at B = 32.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export ROUND=${ROUND:-r04}
bash scripts/gpu/profile.sh c3 c3 || exit 1
BENCH_ARGS_FULL="--gpus 1 --steps 20 --warmup 5" bash scripts/gpu/profile.sh c2 c2 || exit 1
