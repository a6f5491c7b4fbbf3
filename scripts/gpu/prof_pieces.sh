#!/bin/bash
# The one-GPU scaling pieces (scale_pieces.sh) and the kernel stats of the C2
# data-parallel step over a one-rank RCCL group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/scale_pieces.sh || exit 1
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0"
GTR_FORCE_PG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2dp -o run --output-format csv -- \
  python3 bench.py --dp --steps 200 --warmup 20 $LEAN > gpurun_out/c2_dp_rccl1_bench.json 2> gpurun_out/c2_dp.err || { tail -20 gpurun_out/c2_dp.err; exit 1; }
cp "$(find gpurun_out/prof_c2dp -name '*kernel_stats.csv' | head -1)" gpurun_out/c2_dp_rccl1_kernel_stats.csv
rm -rf gpurun_out/prof_c2dp
python3 scripts/kstats.py gpurun_out/c2_dp_rccl1_kernel_stats.csv | head -16
