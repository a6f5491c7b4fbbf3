# all GPU tests, then C2/C3 bench A/B of the chain sweep (+ rocprof stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --maxfail=5 --timeout 150 --timeout-method thread > gpurun_out/t1.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/t1.log | tail -30; tail -60 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for CFG in c2 c3; do
  for CS in 0 1; do
    GTR_CHAIN_SWEEP=$CS timeout -k 10 300 python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/ab_${CFG}_$CS.json 2> gpurun_out/ab_${CFG}_$CS.err || { tail -30 gpurun_out/ab_${CFG}_$CS.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${CFG}_$CS.json')); print('$CFG chain_sweep=$CS', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/prof_$CFG.json 2> gpurun_out/prof_$CFG.err || { tail -30 gpurun_out/prof_$CFG.err; exit 1; }
  python scripts/kstats.py gpurun_out/prof_$CFG/run_kernel_stats.csv
done
