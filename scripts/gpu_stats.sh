set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/st
export TMPDIR=/tmp
for CFG in c2 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st/$CFG -o run -- python3 bench.py --config $CFG --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/st/$CFG.json 2> gpurun_out/st/$CFG.err || { tail -20 gpurun_out/st/$CFG.err; exit 1; }
GTR_GEMM=f32 timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/st/${CFG}_f32.json 2> gpurun_out/st/${CFG}_f32.err || { tail -20 gpurun_out/st/${CFG}_f32.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/st/${CFG}_f32.json')); print('$CFG f32', d['value'], d['ms_per_step'])"
done
find gpurun_out/st -name "*stats.csv"
