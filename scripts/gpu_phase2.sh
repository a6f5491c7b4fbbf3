set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for CFG in c2 c3; do
GTR_LIB=$GRAFT_REPO_ROOT/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python scripts/phase_timing.py --config $CFG > gpurun_out/phase_$CFG.txt 2> gpurun_out/phase_$CFG.err || { tail -30 gpurun_out/phase_$CFG.err; exit 1; }
cat gpurun_out/phase_$CFG.txt
done
