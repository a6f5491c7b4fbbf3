#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
XFLAG= bash scripts/gpu/tests.sh "sort or large_batch" ab11 || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0"
for E in "GTR_SORT=merge" "GTR_SORT=radix"; do
  env $E timeout -k 10 300 python3 bench.py --config c3 --batch-size 8192 --num-batches 8 $LEAN --steps 100 --warmup 10 > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c3 b8192 $E', d['value'], d['ms_per_step'])"
done
GTR_SORT=radix timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab11 -o run --output-format csv -- \
  python3 bench.py --config c3 --batch-size 8192 --num-batches 8 $LEAN --steps 50 --warmup 5 > gpurun_out/ab11_prof.json 2> gpurun_out/ab11_prof.err || { tail -5 gpurun_out/ab11_prof.err; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/prof_ab11 -name '*kernel_stats.csv' | head -1)" | head -20
