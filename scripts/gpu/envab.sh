#!/bin/bash
# A/B of a HIP runtime environment setting on the default C2 line (lean, driver K/W):
# usage: envab.sh "VAR=value" [config]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0 --strong-batches 0 --c1-reps 0"
for r in 1 2 3; do
  for e in "GTR_NOP=1" "$1"; do
    env $e timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config ${2:-c2} $LEAN 2>/dev/null \
      | python3 -c "import json,sys;d=json.load(sys.stdin);print('$e',d['value'],d['ms_per_step'],d['config']['gpu_ms_per_step_events'])" || exit 1
  done
done
