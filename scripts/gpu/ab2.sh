#!/bin/bash
# A/B of the fused begin / tail-with-weight-gradients on the lean C2 bench, the warm/cold
# conv_fwd diagnostic, then the standalone Onesweep sort probe (last: it may fault).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --steps 400 --warmup 30"
for round in 1 2; do
for E in "GTR_TAILW=0" "GTR_TAILW=1" "GTR_TAILW=1 GTR_BEGIN_FUSED=1"; do
  env $E timeout -k 10 300 python3 bench.py --config c2 $LEAN > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c2 $E', d['value'], d['ms_per_step'], d['roofline']['tail_kernel'])"
done
done
for E in "GTR_TAILW=0" "GTR_TAILW=1 GTR_BEGIN_FUSED=1"; do
  env $E timeout -k 10 300 python3 bench.py --config c3 $LEAN > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c3 $E', d['value'], d['ms_per_step'], d['roofline']['tail_kernel'])"
done
GTR_CHAIN_SWEEP=0 GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/dbg_warm.py > gpurun_out/warm.txt 2> gpurun_out/warm.err || { tail -5 gpurun_out/warm.err; exit 1; }
cat gpurun_out/warm.txt
timeout -k 5 60 ./scripts/dbg/onesweep 855000 > gpurun_out/onesweep.txt 2>&1; echo "onesweep rc=$?"; cat gpurun_out/onesweep.txt
