# iteration: GPU parity tests (all), then the large-batch C3 probe with kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --maxfail=5 --timeout 150 --timeout-method thread > gpurun_out/t1.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/t1.log | tail -30; tail -60 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
B=${B:-8192}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_big_$B -o run --output-format csv -- python bench.py --config c3 --batch-size $B --num-batches 8 --steps 50 --warmup 5 --cpu-seconds 0 --recall-steps 0 > gpurun_out/big_prof_$B.json 2> gpurun_out/big_prof_$B.err || { tail -30 gpurun_out/big_prof_$B.err; exit 1; }
cat gpurun_out/big_prof_$B.json
python scripts/kstats.py gpurun_out/prof_big_$B/run_kernel_stats.csv
