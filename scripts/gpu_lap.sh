set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lappe.py -v -m gpu --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/tlap.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/tlap.log | tail; tail -70 gpurun_out/tlap.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/tlap.log | tail -12
timeout -k 10 400 python scripts/lappe_bench.py > gpurun_out/lappe_bench.json 2> gpurun_out/lappe_bench.err || { tail -30 gpurun_out/lappe_bench.err; exit 1; }
cat gpurun_out/lappe_bench.json
