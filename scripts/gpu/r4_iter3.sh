#!/bin/bash
# Round 4 iteration: lazy / sort / sharded parity, C5 B = 1024 kernel stats, and the tail
# window A/B (GTR_TAIL_TW 64 / 128 / 256 builds) on the large-batch lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/tests.sh "sort or lazy or large_batch or sharded or c4 or distributed or c5s" it3 || exit 1
PMC=0 bash scripts/gpu/profile.sh c5 it3_c5_b1024 --batch-size 1024 > /dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/it3_c5_b1024_bench.json'));print('c5_b1024',d['value'],d['ms_per_step'])"
B=/root/repo/gat-recommendation_amd/build
bash scripts/gpu/kbench.sh tw "c5:1024 c3:8192 c5:8192" "GTR_SPLIT=1 GTR_SPLIT=1,GTR_LIB=$B/vTW64/libgtr_hip.so GTR_SPLIT=1,GTR_LIB=$B/vTW256/libgtr_hip.so" > /dev/null
