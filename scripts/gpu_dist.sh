set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -v -m gpu --maxfail=3 --timeout 400 --timeout-method thread > gpurun_out/td.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/td.log | tail; tail -70 gpurun_out/td.log; exit 1; }
grep -E "distributed" gpurun_out/td.log | tail -5; tail -2 gpurun_out/td.log
