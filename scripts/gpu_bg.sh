# GPU batch-constructor tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_batchgen.py -v -m gpu --maxfail=3 --timeout 200 --timeout-method thread > gpurun_out/tbg.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tbg.log | tail; tail -50 gpurun_out/tbg.log; exit 1; }
tail -12 gpurun_out/tbg.log
