# parity tests, then an A/B of an env switch (AB_VAR in {0,1}) with kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VAR=${AB_VAR:-GTR_CONSUMER_REDUCE}
CFG=${CFG:-c2}
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for mode in 0 1; do
env $AB_VAR=$mode timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/ab_$mode -o run --output-format csv -- python bench.py --config $CFG --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || { tail -30 gpurun_out/ab_$mode.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab_$mode.json'));print('$AB_VAR=$mode', d['value'], d['ms_per_step'])"
python scripts/kstats.py gpurun_out/ab_$mode/run_kernel_stats.csv
done
