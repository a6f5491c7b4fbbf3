#!/bin/bash
# Kernel order of the last steps of a short bench run (names, durations, gaps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c4}; EXTRA=${EXTRA:---global-batch 1024}
LEAN="--config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --tail-probe 0 --c1-reps 0 --strong-batches 0 $EXTRA"
rm -rf gpurun_out/tr
GTR_SPLIT=${SPLIT:-1} timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr -o run --output-format csv -- \
  python3 bench.py $LEAN --steps ${TSTEPS:-6} --warmup 4 > gpurun_out/tr_bench.json 2> gpurun_out/tr.err || { tail -20 gpurun_out/tr.err; exit 1; }
f=$(find gpurun_out/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_tail.py "$f" ${NK:-120} > gpurun_out/tr_${CFG}.txt
rm -rf gpurun_out/tr
cat gpurun_out/tr_${CFG}.txt
