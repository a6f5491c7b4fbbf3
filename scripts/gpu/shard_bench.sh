#!/bin/bash
# Row-sharded table on the one-GPU box: RCCL world-1 (graph-captured all-to-alls) against
# the replicated data-parallel step, C2 at B=32 and C5 at B=1024.  Lines under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0"
for CFG in "c2 --batch-size 32" "c5 --batch-size 1024"; do
  for MODE in "--shard-table" "--dp --lazy 1" ""; do
    TAG=$(echo "$CFG $MODE" | tr -c 'a-z0-9' '_')
    GTR_FORCE_PG=1 timeout -k 10 300 python3 bench.py --config $CFG $MODE $LEAN --steps 100 --warmup 10 \
      > gpurun_out/shb_$TAG.json 2> gpurun_out/shb_$TAG.err || { tail -20 gpurun_out/shb_$TAG.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/shb_$TAG.json'));print('$CFG $MODE', d['value'], d['ms_per_step'], d['config']['graph_collectives'], d['config']['parallelism'])"
  done
done
