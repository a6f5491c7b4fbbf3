set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name args
  local N=$1; shift
  timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/nt_$N.json 2> gpurun_out/nt_$N.err || { tail -20 gpurun_out/nt_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/nt_$N.json')); print('$N', d['value'], d['ms_per_step'])"
}
NT=$GRAFT_REPO_ROOT/gat-recommendation_amd/build/nt/libgtr_hip.so
for CFG in c2 c3; do
run ${CFG}_base --config $CFG
GTR_LIB=$NT run ${CFG}_nt --config $CFG
GTR_CHAIN_SWEEP=0 run ${CFG}_nochain --config $CFG
run ${CFG}_base2 --config $CFG
GTR_LIB=$NT run ${CFG}_nt2 --config $CFG
done
