# eval-path GPU tests (score_topk, predict, Recall@K parity)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval.py -v -m gpu --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/te.log 2>&1 || { tail -80 gpurun_out/te.log; exit 1; }
tail -15 gpurun_out/te.log
