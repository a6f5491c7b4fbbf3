set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
b() {  # name env... -- args
  local N=$1; shift
  timeout -k 10 400 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/nts_$N.json 2> gpurun_out/nts_$N.err || { tail -20 gpurun_out/nts_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/nts_$N.json')); print('$N', d['value'], d['ms_per_step'], d['roofline']['traffic'])"
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "large_batch" --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/tnts.log 2>&1 || { tail -30 gpurun_out/tnts.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tnts.log | tail -5
b big_nt --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5
GTR_NO_NT_STORE=1 b big_plain --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5
b c5_nt --config c5 --num-batches 8 --steps 50 --warmup 10
GTR_NO_NT_STORE=1 b c5_plain --config c5 --num-batches 8 --steps 50 --warmup 10
b c2 --config c2
