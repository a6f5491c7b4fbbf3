#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GTR_CHAIN_SWEEP=0 GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/dbg_warm.py > gpurun_out/warm.txt 2> gpurun_out/warm.err || { tail -20 gpurun_out/warm.err; exit 1; }
cat gpurun_out/warm.txt
LEAN="--config c2 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0 --steps 400 --warmup 30"
for R in "" "--resident"; do
  timeout -k 10 300 python3 bench.py $LEAN $R > gpurun_out/res.json 2>> gpurun_out/res.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/res.json'));print('resident=$R', d['value'], d['ms_per_step'], d['config']['gpu_ms_per_step_events'])"
done
