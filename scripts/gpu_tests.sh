# all GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -80 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
