#!/bin/bash
# The round's profile set on one MI355X (kernel stats, PMC traffic and the bench line of
# each configuration from the same tree and box; copy gpurun_out/<cfg>_* to profiles/rNN/).
# usage: final_profiles.sh [configs...]   default: every configuration below
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export ROUND=${ROUND:-r06}
ALL="c2 c3_b8192 c4_b1024_split c4_b1024 c4_b8192 c5 c5_b1024"
for c in ${@:-$ALL}; do
  case $c in
    c2) BENCH_ARGS_FULL="--gpus 1 --steps 20 --warmup 5" bash scripts/gpu/profile.sh c2 c2 || exit 1 ;;
    c3_b8192) bash scripts/gpu/profile.sh c3 c3_b8192 --batch-size 8192 || exit 1 ;;
    c4_b1024_split) GTR_SPLIT=1 bash scripts/gpu/profile.sh c4 c4_b1024_split --global-batch 1024 || exit 1 ;;
    c4_b1024) bash scripts/gpu/profile.sh c4 c4_b1024 --global-batch 1024 || exit 1 ;;
    c4_b8192) bash scripts/gpu/profile.sh c4 c4_b8192 --global-batch 8192 || exit 1 ;;
    c5) bash scripts/gpu/profile.sh c5 c5 || exit 1 ;;  # B = 8192 (the c5 default)
    c5_b1024) bash scripts/gpu/profile.sh c5 c5_b1024 --batch-size 1024 || exit 1 ;;
    *) echo "unknown config $c"; exit 1 ;;
  esac
done
