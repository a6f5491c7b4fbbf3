set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
GTR_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --global-batch 64 --steps 30 --warmup 5 > gpurun_out/dp2s.json 2> gpurun_out/dp2s.err || { grep -v "^W2026\|^I2026" gpurun_out/dp2s.err | tail -40; exit 1; }
cat gpurun_out/dp2s.json
