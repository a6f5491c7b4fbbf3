# GPU: parity + DP tests, torchrun N=1 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1 || { tail -80 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_tr1.json 2> gpurun_out/bench_tr1.err || { tail -30 gpurun_out/bench_tr1.err; exit 1; }
cat gpurun_out/bench_tr1.json
