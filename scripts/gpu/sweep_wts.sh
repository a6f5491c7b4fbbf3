#!/bin/bash
# C2 sweep-slice weights A/B (GTR_SWEEP_WTS: conv_fwd(l).., readout, conv_bwd(L-1)..0); WTS="..." overrides the list.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps 400 --warmup 20"
for rep in 1 2; do
for w in ${WTS:-"" "0,1,0.75,1,1" "0,0.75,0.75,1.25,1"}; do
  if [ -z "$w" ]; then unset GTR_SWEEP_WTS; else export GTR_SWEEP_WTS=$w; fi
  timeout -k 10 120 python3 bench.py $LEAN > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw.json'));print('${w:-default}', d['ms_per_step'])"
done; done
