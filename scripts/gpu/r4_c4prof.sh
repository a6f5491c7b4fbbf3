#!/bin/bash
# Round 4: kernel stats of the sharded C4 step at world 1, per-rank B = 1024 and 8192,
# plus the drop-in FFN epoch test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --c1-reps 0 --tail-probe 0 --strong-batches 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k ffn > gpurun_out/t_ffn.log 2>&1 || { tail -30 gpurun_out/t_ffn.log; exit 1; }
tail -3 gpurun_out/t_ffn.log
for GB in 1024 8192; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_$GB -o run --output-format csv -- \
    python3 bench.py --config c4 --global-batch $GB --steps 50 --warmup 10 $LEAN > gpurun_out/c4_b${GB}_bench.json \
    2> gpurun_out/c4_b${GB}.err || { tail -20 gpurun_out/c4_b${GB}.err; exit 1; }
  cp "$(find gpurun_out/prof_c4_$GB -name '*kernel_stats.csv' | head -1)" gpurun_out/c4_b${GB}_kernel_stats.csv
  rm -rf gpurun_out/prof_c4_$GB
  python3 scripts/kstats.py gpurun_out/c4_b${GB}_kernel_stats.csv
  cat gpurun_out/c4_b${GB}_bench.json | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['ms_per_step'])"
done
