set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/bst -o run --output-format csv -- python bench.py --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/bst.json 2> gpurun_out/bst.err || { tail -20 gpurun_out/bst.err; exit 1; }
rm -f gpurun_out/bst/run_kernel_trace.csv
python scripts/kstats.py gpurun_out/bst/run_kernel_stats.csv | head -14
