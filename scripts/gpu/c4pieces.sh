#!/bin/bash
# The sharded C4 step at world 1: the global batch 8192 (N = 1 point of the strong curve)
# and 1024 sessions (the per-rank batch at N = 8) on the split layer path SyncBN runs there.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0"
run() { local tag=$1; shift; timeout -k 10 400 "$@" > gpurun_out/sp_$tag.json 2> gpurun_out/sp_$tag.err || { tail -20 gpurun_out/sp_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sp_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['config']['parallelism'], d['config'].get('step_graph'))"; }
run c4_8192 python3 bench.py --config c4 --steps 100 --warmup 10 $LEAN
GTR_SPLIT=1 run c4_1024_split python3 bench.py --config c4 --global-batch 1024 --steps 200 --warmup 20 $LEAN
run c4_1024 python3 bench.py --config c4 --global-batch 1024 --steps 200 --warmup 20 $LEAN
