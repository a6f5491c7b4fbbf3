# C5-scale single-GPU point (1M items, 9M edges, d=128, B=8192) + kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_c5 -o run --output-format csv -- python bench.py --config c5 --num-batches 4 --steps 30 --warmup 5 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -30 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
python scripts/kstats.py gpurun_out/prof_c5/run_kernel_stats.csv
