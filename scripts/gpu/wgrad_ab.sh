#!/bin/bash
# Weight gradients on MFMA tiles: parity of the large-batch paths, then A/B against the VALU tiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
GTR_WGRAD=mfma XFLAG= bash scripts/gpu/tests.sh "large_batch or grads or fused_steps or c3_large" wgrad_mfma || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0"
for E in "GTR_WGRAD=valu" "GTR_WGRAD=mfma"; do
  env $E timeout -k 10 300 python3 bench.py --config c3 --batch-size 8192 --num-batches 8 $LEAN --steps 100 --warmup 10 > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c3 b8192 $E', d['value'], d['ms_per_step'])"
done
for E in "GTR_WGRAD=valu" "X=1" "GTR_WGRAD=valu" "X=1"; do
  env $E timeout -k 10 300 python3 bench.py --config c2 $LEAN --steps 400 --warmup 30 > gpurun_out/v.json 2>> gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('c2 $E', d['value'], d['ms_per_step'])"
done
GTR_WGRAD=mfma timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wg -o run --output-format csv -- \
  python3 bench.py --config c3 --batch-size 8192 --num-batches 8 $LEAN --steps 50 --warmup 10 > /dev/null 2> gpurun_out/prof_wg.err || exit 1
python3 scripts/kstats.py "$(find gpurun_out/prof_wg -name '*kernel_stats.csv' | head -1)" | head -16
