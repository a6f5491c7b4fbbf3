set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 || { grep -E "FAIL|ERROR" gpurun_out/t1.log | head -20; tail -40 gpurun_out/t1.log; exit 1; }
tail -1 gpurun_out/t1.log
b() {  # name args
  local N=$1; shift
  timeout -k 10 400 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/big_$N.json 2> gpurun_out/big_$N.err || { tail -20 gpurun_out/big_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/big_$N.json')); print('$N', d['value'], d['ms_per_step'], d['roofline']['frac'])"
}
b c2 --config c2
b c3 --config c3
b c3_b8192 --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5
b c5 --config c5 --num-batches 8 --steps 50 --warmup 10
GTR_LIB=$GRAFT_REPO_ROOT/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python scripts/phase_timing.py --config c3 --batch-size 8192 --steps 5 > gpurun_out/phase_big.txt 2> gpurun_out/phase_big.err || { tail -5 gpurun_out/phase_big.err; exit 1; }
cat gpurun_out/phase_big.txt
