#!/bin/bash
# Bench-line A/B over environment settings (lean C2 lines unless CFG / BARGS say otherwise).
# usage: scripts/gpu/envab.sh TAG "ENV1" "ENV2" ...   (each ENVi: space-separated VAR=VALUE, or "-")
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
LEAN="--config ${CFG:-c2} --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --c1-reps 0 --tail-probe 0 --steps ${STEPS:-300} --warmup 30 ${BARGS:-}"
O=gpurun_out/${TAG}_envab.txt
: > $O
for rep in 1 2; do
  for e in "$@"; do
    E=""; [ "$e" != "-" ] && E="$e"
    env $E timeout -k 10 300 python3 bench.py $LEAN > gpurun_out/${TAG}_x.json 2> gpurun_out/${TAG}_x.err || { tail -20 gpurun_out/${TAG}_x.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_x.json'));print(sys.argv[1], d['ms_per_step'], d['config']['gpu_ms_per_step_events'], d['value'])" "[$e]" >> $O
  done
done
cat $O
