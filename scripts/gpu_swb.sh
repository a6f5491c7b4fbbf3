set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for CFG in c2 c3; do
for SB in 64 128 192 256; do
GTR_SWEEP_BLOCKS=$SB timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/swb_${CFG}_$SB.json 2> gpurun_out/swb_${CFG}_$SB.err || { tail -20 gpurun_out/swb_${CFG}_$SB.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/swb_${CFG}_$SB.json')); print('$CFG blocks=$SB', d['value'], d['ms_per_step'])"
done
GTR_CHAIN_SWEEP=0 timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/swb_${CFG}_off.json 2> gpurun_out/swb_${CFG}_off.err || { tail -20 gpurun_out/swb_${CFG}_off.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/swb_${CFG}_off.json')); print('$CFG chain off', d['value'], d['ms_per_step'], d['roofline']['tail_kernel'])"
done
