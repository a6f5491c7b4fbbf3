# pipeline tests + 2-rank bench rehearsal on one GPU (gloo transport, both ranks on cuda:0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/tp.log 2>&1 || { tail -60 gpurun_out/tp.log; exit 1; }
tail -3 gpurun_out/tp.log
GTR_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { tail -40 gpurun_out/dp2.err; exit 1; }
cat gpurun_out/dp2.json
