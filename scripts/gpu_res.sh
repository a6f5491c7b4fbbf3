set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "resident or dropout_deterministic" --maxfail=3 --timeout 200 --timeout-method thread > gpurun_out/tres.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tres.log | tail; tail -40 gpurun_out/tres.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tres.log | tail -4
for CFG in c2 c3; do
for M in res copy; do
X=""; [ $M = copy ] && X="--copy-blob"
timeout -k 10 300 python bench.py --config $CFG $X --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/res_${CFG}_$M.json 2> gpurun_out/res_${CFG}_$M.err || { tail -20 gpurun_out/res_${CFG}_$M.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/res_${CFG}_$M.json')); print('$CFG $M', d['value'], d['ms_per_step'], d['config']['gpu_ms_per_step_events'])"
done
done
