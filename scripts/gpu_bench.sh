# smoke + bench + rocprofv3 kernel-trace summary (round profile)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c2}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log | tail -20; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --config $CFG --steps 300 --warmup 30 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err || { tail -30 gpurun_out/bench_$CFG.err; exit 1; }
cat gpurun_out/bench_$CFG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/bench_prof_$CFG.json 2> gpurun_out/bench_prof_$CFG.err || { tail -30 gpurun_out/bench_prof_$CFG.err; exit 1; }
find gpurun_out/prof_$CFG -name "*stats*" | head
