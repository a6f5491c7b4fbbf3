#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
XFLAG= bash scripts/gpu/tests.sh "parity or fullsize or lagged or lazy" ab9 || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --steps 400 --warmup 30"
for round in 1 2; do
for E in "GTR_SWEEP_BLOCKS=128" "GTR_SWEEP_BLOCKS=0"; do
for C in c2 c3; do
  env $E timeout -k 10 300 python3 bench.py --config $C $LEAN > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('$C $E', d['value'], d['ms_per_step'])"
done
done
done
