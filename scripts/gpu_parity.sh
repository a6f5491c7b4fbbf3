set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1
rc=$?
tail -30 gpurun_out/t1.log
exit $rc
