#!/bin/bash
# Iteration check: full GPU suite (no -x), then A/B of row-group widths on C2 / C3 and the
# C3 B = 8192 lean line.  Logs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
XFLAG= bash scripts/gpu/tests.sh "" iter || exit 1
bash scripts/gpu/ab.sh c2 GTR_ROW_GROUP=16 GTR_ROW_GROUP=12 GTR_ROW_GROUP=8 || exit 1
bash scripts/gpu/ab.sh c3 GTR_ROW_GROUP=16 GTR_ROW_GROUP=12 GTR_ROW_GROUP=8 || exit 1
timeout -k 10 300 python3 bench.py --config c3 --batch-size 8192 --num-batches 8 --cpu-seconds 0 --gather-batch 0 \
  --recall-steps 0 --e2e-steps 0 --tail-probe 0 --steps 100 --warmup 10 > gpurun_out/iter_b8192.json 2> gpurun_out/iter_b8192.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/iter_b8192.json'));print('c3 b8192', d['value'], d['ms_per_step'])"
