#!/bin/bash
# One-GPU pieces of the strong-scaling projection: the sharded C4 / C5 steps at world 1 at
# the global batch (N = 1 point) and at the per-rank batch of N = 8 (1024), and the C2
# data-parallel step over a one-rank RCCL group (the exchange path at world 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0"
run() { local tag=$1; shift; timeout -k 10 400 "$@" > gpurun_out/sp_$tag.json 2> gpurun_out/sp_$tag.err || { tail -20 gpurun_out/sp_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sp_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['config']['parallelism'], d['config'].get('dp_exchange'))"; }
run c5s_8192 python3 bench.py --config c5s --steps 30 --warmup 5 $LEAN
run c5s_1024 python3 bench.py --config c5s --global-batch 1024 --steps 50 --warmup 10 $LEAN
run c4_8192 python3 bench.py --config c4 --steps 30 --warmup 5 $LEAN
run c4_1024 python3 bench.py --config c4 --global-batch 1024 --steps 50 --warmup 10 $LEAN
GTR_FORCE_PG=1 run c2_dp_rccl1 python3 bench.py --dp --steps 200 --warmup 20 $LEAN
