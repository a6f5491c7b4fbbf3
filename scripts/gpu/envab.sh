#!/bin/bash
# A/B of environment settings on one bench line (lean, driver K/W), three alternating rounds:
# usage: envab.sh "VAR=value[,VAR=value] ..." [bench args...]   (first variant = baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --tail-probe 0 --strong-batches 0 --c1-reps 0"
VARS=$1; shift
EXTRA=${*:---config c2}
for r in 1 2 3; do
  for e in GTR_NOP=1 $VARS; do
    env ${e//,/ } timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $EXTRA $LEAN 2>/dev/null \
      | python3 -c "import json,sys;d=json.load(sys.stdin);print('$e',d['value'],d['ms_per_step'],d['config']['gpu_ms_per_step_events'])" || exit 1
  done
done
