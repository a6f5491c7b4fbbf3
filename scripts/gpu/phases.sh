#!/bin/bash
# Per-workgroup phase stamps of the layer kernels (timing build, no XCD packing), C2 and C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for CFG in c2 c3; do
  GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --config $CFG --steps 30 \
    > gpurun_out/phases_$CFG.txt 2> gpurun_out/phases_$CFG.err || { tail -20 gpurun_out/phases_$CFG.err; exit 1; }
  cat gpurun_out/phases_$CFG.txt
done
