set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
b() {  # cfg name env...
  local CFG=$1 N=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/swc_${CFG}_$N.json 2> gpurun_out/swc_${CFG}_$N.err || { tail -20 gpurun_out/swc_${CFG}_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/swc_${CFG}_$N.json')); print('$CFG $N', d['value'], d['ms_per_step'])"
}
for CFG in c2 c3; do
for SB in 96 112 128 144 160; do b $CFG b$SB GTR_SWEEP_BLOCKS=$SB; done
b $CFG b128_w11111 GTR_SWEEP_BLOCKS=128 GTR_SWEEP_WTS=1,1,1,1,1
b $CFG b128_w11511 GTR_SWEEP_BLOCKS=128 GTR_SWEEP_WTS=1,1,0.5,1,1
b $CFG b128_w12121 GTR_SWEEP_BLOCKS=128 GTR_SWEEP_WTS=1,1.2,0.75,1.2,1
done
