set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "lazy or lagged" --maxfail=3 --timeout 200 --timeout-method thread > gpurun_out/tlag.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tlag.log | tail; tail -60 gpurun_out/tlag.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tlag.log | tail -14
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -v -m gpu --maxfail=3 --timeout 400 --timeout-method thread > gpurun_out/tlagd.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tlagd.log | tail; tail -60 gpurun_out/tlagd.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tlagd.log | tail -6
run() {  # name args
  local N=$1; shift
  timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/lag_$N.json 2> gpurun_out/lag_$N.err || { tail -20 gpurun_out/lag_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lag_$N.json')); print('$N', d['value'], d['ms_per_step'])"
}
run c2_eager --lagged 0
run c2_lagged --lagged 1
run c2_dp_eager --dp --lagged 0
run c2_dp_lagged --dp --lagged 1
run c3_eager --config c3 --lagged 0
run c3_lagged --config c3 --lagged 1
run c3_dp_eager --config c3 --dp --lagged 0
run c3_dp_lagged --config c3 --dp --lagged 1
