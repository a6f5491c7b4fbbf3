# A/B: sweep beside the chain vs serial (kernel stats of both)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for mode in 0 1; do
GTR_SERIAL_SWEEP=$mode timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/exp_$mode -o run --output-format csv -- python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/exp_$mode.json 2> gpurun_out/exp_$mode.err || { tail -30 gpurun_out/exp_$mode.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/exp_$mode.json'));print('serial=$mode', d['value'], d['ms_per_step'])"
python scripts/kstats.py gpurun_out/exp_$mode/run_kernel_stats.csv
done
