# parity + phase stamps (C2, C3) + bench (C2, C3), no profiler
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1 || { tail -60 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for CFG in c2 c3; do
  CFG=$CFG bash scripts/gpu_phase.sh || exit 1
  timeout -k 10 600 python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err || { tail -30 gpurun_out/bench_$CFG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$CFG.json'));print('$CFG', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
