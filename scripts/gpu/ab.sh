#!/bin/bash
# A/B of environment settings on the lean bench: scripts/gpu/ab.sh CFG "ENV_A" "ENV_B" [...]
# (AB_EXTRA: extra bench args for every setting)
# prints value / ms_per_step per setting (two alternating rounds), log under gpurun_out/ab_*.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CFG=$1; shift
for round in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python3 bench.py --config $CFG --steps 400 --warmup 30 --cpu-seconds 0 --gather-batch 0 \
      --recall-steps 0 --e2e-steps 0 --tail-probe 0 ${AB_EXTRA:-} > gpurun_out/ab_out.json 2>> gpurun_out/ab_err.log || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_out.json'));print('$CFG', '$e', d['value'], d['ms_per_step'])" | tee -a gpurun_out/ab_${CFG}.log
  done
done
