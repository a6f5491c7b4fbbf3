# large-batch probes (gather-family roofline): C3 at B=1024 and B=8192, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 1024 8192; do
  timeout -k 10 300 python bench.py --config c3 --batch-size $B --num-batches 8 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/big_$B.json 2> gpurun_out/big_$B.err || { tail -30 gpurun_out/big_$B.err; exit 1; }
  cat gpurun_out/big_$B.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_big_$B -o run --output-format csv -- python bench.py --config c3 --batch-size $B --num-batches 8 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/big_prof_$B.json 2> gpurun_out/big_prof_$B.err || { tail -30 gpurun_out/big_prof_$B.err; exit 1; }
  python scripts/kstats.py gpurun_out/prof_big_$B/run_kernel_stats.csv
done
