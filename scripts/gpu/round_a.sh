#!/bin/bash
# Round-2 artifacts, part A: C2 (the headline, full bench line) and C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
BENCH_ARGS_FULL="--config c2" bash scripts/gpu/profile.sh c2 c2 || exit 1
bash scripts/gpu/profile.sh c3 c3 || exit 1
