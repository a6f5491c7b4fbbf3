# full round measurement: parity, smoke, phase stamps, bench (+CPU baseline), rocprof stats for C2 and C3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1 || { tail -60 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
CFG=c2 bash scripts/gpu_phase.sh || exit 1
for CFG in c2 c3; do
  CPUS=0; [ $CFG = c2 ] && CPUS=15
  timeout -k 10 600 python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds $CPUS > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err || { tail -30 gpurun_out/bench_$CFG.err; exit 1; }
  cat gpurun_out/bench_$CFG.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/bench_prof_$CFG.json 2> gpurun_out/bench_prof_$CFG.err || { tail -30 gpurun_out/bench_prof_$CFG.err; exit 1; }
  python scripts/kstats.py gpurun_out/prof_$CFG/run_kernel_stats.csv
done
