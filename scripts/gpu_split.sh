set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/ts.log 2>&1 || { grep -E "FAIL|ERROR" gpurun_out/ts.log | head -20; grep -E "relative error|Mismatch|assert" gpurun_out/ts.log | head -20; tail -30 gpurun_out/ts.log; exit 1; }
tail -1 gpurun_out/ts.log
for CFG in c2 c3; do
for G in split f32; do
GTR_GEMM=$G timeout -k 10 300 python bench.py --config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/sp_${CFG}_$G.json 2> gpurun_out/sp_${CFG}_$G.err || { tail -20 gpurun_out/sp_${CFG}_$G.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sp_${CFG}_$G.json')); print('$CFG $G', d['value'], d['ms_per_step'], d['config']['final_loss'])"
done
GTR_LIB=$GRAFT_REPO_ROOT/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python scripts/phase_timing.py --config $CFG > gpurun_out/phase_$CFG.txt 2> gpurun_out/phase_$CFG.err || { tail -30 gpurun_out/phase_$CFG.err; exit 1; }
cat gpurun_out/phase_$CFG.txt
done
