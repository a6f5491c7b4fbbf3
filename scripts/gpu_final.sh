# default bench lines of the round (each as the driver runs it, plus c3 / c5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-v8}
timeout -k 10 600 python bench.py > gpurun_out/c2_${V}_bench.json 2> gpurun_out/c2_${V}_bench.err || { tail -30 gpurun_out/c2_${V}_bench.err; exit 1; }
cat gpurun_out/c2_${V}_bench.json
timeout -k 10 600 python bench.py --config c3 > gpurun_out/c3_${V}_bench.json 2> gpurun_out/c3_${V}_bench.err || { tail -30 gpurun_out/c3_${V}_bench.err; exit 1; }
cat gpurun_out/c3_${V}_bench.json
timeout -k 10 600 python bench.py --config c5 --num-batches 8 --steps 50 --warmup 10 --recall-steps 0 --e2e-steps 0 --gather-batch 0 --cpu-seconds 0 > gpurun_out/c5_${V}_bench.json 2> gpurun_out/c5_${V}_bench.err || { tail -30 gpurun_out/c5_${V}_bench.err; exit 1; }
cat gpurun_out/c5_${V}_bench.json
