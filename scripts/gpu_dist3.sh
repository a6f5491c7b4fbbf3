set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -v -m gpu --maxfail=3 --timeout 400 --timeout-method thread > gpurun_out/td3.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/td3.log | tail; tail -70 gpurun_out/td3.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/td3.log | tail -6
GTR_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/dp2s.json 2> gpurun_out/dp2s.err || { grep -v "^W2026\|^I2026" gpurun_out/dp2s.err | tail -40; exit 1; }
wc -l gpurun_out/dp2s.json
python -c "import json; d=json.load(open('gpurun_out/dp2s.json')); print('2 ranks shared', d['value'], d['config']['replicas_identical'], d['config']['lagged_sweep'])"
GTR_FORCE_PG=1 timeout -k 10 300 python bench.py --dp --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/rccl1.json 2> gpurun_out/rccl1.err || { tail -30 gpurun_out/rccl1.err; exit 1; }
wc -l gpurun_out/rccl1.json
python -c "import json; d=json.load(open('gpurun_out/rccl1.json')); print('rccl world1', d['value'], d['ms_per_step'], d['config']['graph_collectives'], d['config']['lagged_sweep'])"
