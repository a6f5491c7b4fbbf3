#!/bin/bash
# k_lazy_catchup slots-per-wave sweep at C5 (B = 1024 and 8192): bench ms/step per setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--config c5 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --c1-reps 0 --tail-probe 0 --steps 100 --warmup 20"
for B in 1024 8192; do
  for S in ${SPWS:-1 2 4 8 16 32 64}; do
    GTR_CATCHUP_SPW=$S timeout -k 10 200 python3 bench.py $LEAN --batch-size $B > gpurun_out/cu_${B}_$S.json 2> gpurun_out/cu_${B}_$S.err \
      || { tail -20 gpurun_out/cu_${B}_$S.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/cu_${B}_$S.json'));print('B=$B spw=$S', d['ms_per_step'])"
  done
done
