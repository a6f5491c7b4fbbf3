# phase stamps of the layer kernels (timing build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c2}
GTR_LIB=$GRAFT_REPO_ROOT/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python scripts/phase_timing.py --config $CFG ${PH_ARGS:-} > gpurun_out/phase_$CFG.txt 2> gpurun_out/phase_$CFG.err || { tail -30 gpurun_out/phase_$CFG.err; exit 1; }
cat gpurun_out/phase_$CFG.txt
