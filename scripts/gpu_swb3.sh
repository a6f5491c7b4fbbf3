set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
b() {  # cfg name env...
  local CFG=$1 N=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/swd_${CFG}_$N.json 2> gpurun_out/swd_${CFG}_$N.err || { tail -20 gpurun_out/swd_${CFG}_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/swd_${CFG}_$N.json')); print('$CFG $N', d['value'], d['ms_per_step'])"
}
for SB in 96 128 160 192; do b c2 b$SB GTR_SWEEP_BLOCKS=$SB; done
b c2 w1 GTR_SWEEP_WTS=1,1,1,1,1
b c2 w_fwd_heavy GTR_SWEEP_WTS=1.2,1.2,0.6,1,1
b c2 w_bwd_heavy GTR_SWEEP_WTS=0.8,0.8,0.6,1.2,1.2
b c2 b128again GTR_SWEEP_BLOCKS=128
