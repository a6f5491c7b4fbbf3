# quick: GPU parity tests + phase stamps + bench (no profiler)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c2}
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 -x > gpurun_out/t1.log 2>&1 || { tail -60 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
bash scripts/gpu_phase.sh
timeout -k 10 600 python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err || { tail -30 gpurun_out/bench_$CFG.err; exit 1; }
cat gpurun_out/bench_$CFG.json
