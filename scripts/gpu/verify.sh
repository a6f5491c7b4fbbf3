#!/bin/bash
# Round-2 verification: full GPU suite on the defaults, the opt-in paths on their tests
# (GTR_TAILW=1: tail with in-launch weight gradients; GTR_BEGIN_FUSED=1: step begin inside
# conv_fwd(0); GTR_SORT=onesweep: large-batch sort), then A/B bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
XFLAG= bash scripts/gpu/tests.sh "" full || exit 1
GTR_TAILW=1 GTR_BEGIN_FUSED=1 bash scripts/gpu/tests.sh "parity or fullsize or distributed or dropin or pipeline or sharded" fused || exit 1
GTR_SORT=onesweep bash scripts/gpu/tests.sh "large_batch or 2100 or capacity" onesweep || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --steps 400 --warmup 30"
for E in "GTR_TAILW=0" "GTR_TAILW=1" "GTR_TAILW=1 GTR_BEGIN_FUSED=1"; do
  env $E timeout -k 10 300 python3 bench.py --config c2 $LEAN > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c2 $E', d['value'], d['ms_per_step'], d['roofline']['tail_kernel'])"
done
for E in "GTR_SORT=merge" "GTR_SORT=onesweep"; do
  env $E timeout -k 10 300 python3 bench.py --config c3 --batch-size 8192 --num-batches 8 $LEAN --steps 100 --warmup 10 > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c3 b8192 $E', d['value'], d['ms_per_step'])"
done
