#!/bin/bash
# Round 4 iteration: sort / lazy / sharded parity, then kernel stats (no PMC) of the
# per-rank small-batch lines (C5 B = 1024 lazy, C4 B = 1024 sharded split path).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export ROUND=r04
bash scripts/gpu/tests.sh "sort or lazy or large_batch or sharded or c4 or distributed or c5s" it2 || exit 1
PMC=0 bash scripts/gpu/profile.sh c5 it2_c5_b1024 --batch-size 1024 > /dev/null || exit 1
GTR_SPLIT=1 PMC=0 bash scripts/gpu/profile.sh c4 it2_c4_b1024 --global-batch 1024 > /dev/null || exit 1
for t in it2_c5_b1024 it2_c4_b1024; do python3 -c "import json;d=json.load(open('gpurun_out/${t}_bench.json'));print('$t',d['value'],d['ms_per_step'])"; done
