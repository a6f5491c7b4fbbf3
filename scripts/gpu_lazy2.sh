set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "lazy" --maxfail=3 --timeout 200 --timeout-method thread > gpurun_out/tl.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tl.log | tail; tail -60 gpurun_out/tl.log; exit 1; }
tail -2 gpurun_out/tl.log
run() {  # name args
  local N=$1; shift
  timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/ab_$N.json 2> gpurun_out/ab_$N.err || { tail -20 gpurun_out/ab_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$N.json')); print('$N', d['value'], d['ms_per_step'])"
}
run c2_lazy --config c2 --lazy 1
run c5b1k_eager --config c5 --batch-size 1024 --num-batches 8 --steps 50 --warmup 10 --lazy 0
run c5b1k_lazy --config c5 --batch-size 1024 --num-batches 8 --steps 50 --warmup 10 --lazy 1
run c5b256_eager --config c5 --batch-size 256 --num-batches 16 --steps 100 --warmup 20 --lazy 0
run c5b256_lazy --config c5 --batch-size 256 --num-batches 16 --steps 100 --warmup 20 --lazy 1
run c5_lazy --config c5 --num-batches 4 --steps 30 --warmup 5 --lazy 1
