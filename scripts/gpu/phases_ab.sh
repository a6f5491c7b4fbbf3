#!/bin/bash
# Phase stamps of the C2 step under sweep variants (timing build, no XCD packing).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for E in "GTR_CHAIN_SWEEP=0" "GTR_SWEEP_BLOCKS=32" "GTR_SWEEP_BLOCKS=96"; do
  echo "== $E"
  env $E GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --config c2 --steps 30 \
    > gpurun_out/phases_ab.txt 2> gpurun_out/phases_ab.err || { tail -20 gpurun_out/phases_ab.err; exit 1; }
  cat gpurun_out/phases_ab.txt
done
bash scripts/gpu/ab.sh c2 GTR_SWEEP_BLOCKS=0 GTR_SWEEP_BLOCKS=32 GTR_SWEEP_BLOCKS=64
