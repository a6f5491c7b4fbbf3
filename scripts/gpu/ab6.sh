#!/bin/bash
# Kernel stats of the current C2 step (rocprofv3) + A/B resident images / fused begin.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab6 -o run --output-format csv -- \
  python3 bench.py --config c2 $LEAN --steps 200 --warmup 20 > gpurun_out/ab6_prof.json 2> gpurun_out/ab6_prof.err || { tail -5 gpurun_out/ab6_prof.err; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/prof_ab6 -name '*kernel_stats.csv' | head -1)"
LEAN="$LEAN --steps 400 --warmup 30"
for round in 1 2; do
for E in "--resident" "" ; do
for F in "GTR_BEGIN_FUSED=0" "GTR_BEGIN_FUSED=1"; do
  env $F timeout -k 10 300 python3 bench.py --config c2 $LEAN $E > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c2 $E $F', d['value'], d['ms_per_step'], d['config']['gpu_ms_per_step_events'])"
done
done
done
