set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python scripts/lappe_bench.py > gpurun_out/lappe_bench.json 2> gpurun_out/lappe_bench.err || { tail -30 gpurun_out/lappe_bench.err; exit 1; }
cat gpurun_out/lappe_bench.json
timeout -k 10 400 python bench.py --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/c3_b8192_v8_bench.json 2> gpurun_out/c3_b8192_v8_bench.err || { tail -30 gpurun_out/c3_b8192_v8_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c3_b8192_v8_bench.json')); print('c3 b8192', d['value'], d['ms_per_step'], d['roofline']['frac'])"
