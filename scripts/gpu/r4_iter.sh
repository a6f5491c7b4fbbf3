#!/bin/bash
# Round 4 iteration: a -k subset of the GPU tests, then kernel stats of the sharded C4 step
# at world 1 (per-rank B = 1024 and 8192).  usage: r4_iter.sh "<pytest -k expr>" [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-sharded}
TAG=${2:-it}
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --c1-reps 0 --tail-probe 0 --strong-batches 0"
if [ "$K" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "$K" > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
  tail -3 gpurun_out/t_$TAG.log
fi
for GB in ${GBS:-1024 8192}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_$GB -o run --output-format csv -- \
    python3 bench.py --config c4 --global-batch $GB --steps 50 --warmup 10 $LEAN > gpurun_out/${TAG}_c4_b${GB}_bench.json \
    2> gpurun_out/${TAG}_c4_b${GB}.err || { tail -20 gpurun_out/${TAG}_c4_b${GB}.err; exit 1; }
  cp "$(find gpurun_out/prof_c4_$GB -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_c4_b${GB}_kernel_stats.csv
  rm -rf gpurun_out/prof_c4_$GB
  python3 scripts/kstats.py gpurun_out/${TAG}_c4_b${GB}_kernel_stats.csv
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_c4_b${GB}_bench.json'));print('c4',$GB,d['value'],d['ms_per_step'])"
done
