set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 || { grep -E "FAIL|ERROR" gpurun_out/t1.log | head -20; tail -60 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for CFG in c2 c3; do
timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/kx_$CFG.json 2> gpurun_out/kx_$CFG.err || { tail -20 gpurun_out/kx_$CFG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/kx_$CFG.json')); print('$CFG', d['value'], d['ms_per_step'])"
GTR_LIB=$GRAFT_REPO_ROOT/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python scripts/phase_timing.py --config $CFG > gpurun_out/phase_$CFG.txt 2> gpurun_out/phase_$CFG.err || { tail -30 gpurun_out/phase_$CFG.err; exit 1; }
cat gpurun_out/phase_$CFG.txt
done
