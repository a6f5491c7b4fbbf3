#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --steps 400 --warmup 30"
for round in 1 2; do
for E in "GTR_SWEEP_BLOCKS=128" "GTR_SWEEP_BLOCKS=224" "GTR_SWEEP_BLOCKS=256" "GTR_SWEEP_BLOCKS=256 GTR_SWEEP_WTS=0,1,1,1,1"; do
  env $E timeout -k 10 300 python3 bench.py --config c2 $LEAN > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c2 $E', d['value'], d['ms_per_step'])"
done
done
