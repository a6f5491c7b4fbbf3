#!/bin/bash
# A/B of the row-group width (GTR_ROW_GROUP) at C2, C3 and C3 B = 8192.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/gpu/ab.sh c2 GTR_ROW_GROUP=8 GTR_ROW_GROUP=6 GTR_ROW_GROUP=4 || exit 1
bash scripts/gpu/ab.sh c3 GTR_ROW_GROUP=8 GTR_ROW_GROUP=6 GTR_ROW_GROUP=4 || exit 1
for R in 16 12 8; do
  GTR_ROW_GROUP=$R timeout -k 10 300 python3 bench.py --config c3 --batch-size 8192 --num-batches 8 --cpu-seconds 0 --gather-batch 0 \
    --recall-steps 0 --e2e-steps 0 --tail-probe 0 --steps 100 --warmup 10 > gpurun_out/rg_b8192.json 2>> gpurun_out/rg_b8192.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/rg_b8192.json'));print('c3 b8192 R=$R', d['value'], d['ms_per_step'])"
done
