set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -k "dp or lazy or lagged or distributed or rccl" -v -m gpu --maxfail=3 --timeout 400 --timeout-method thread > gpurun_out/tdp3.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tdp3.log | tail; tail -50 gpurun_out/tdp3.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tdp3.log | tail -14
for M in 0 1; do
GTR_FORCE_PG=1 GTR_GRAPH_COLL=1 timeout -k 10 300 python bench.py --dp --lagged $M --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/dp3_$M.json 2> gpurun_out/dp3_$M.err || { tail -20 gpurun_out/dp3_$M.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dp3_$M.json')); print('rccl dp lagged=$M', d['value'], d['ms_per_step'], d['roofline']['tail_kernel'])"
done
