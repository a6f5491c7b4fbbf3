set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "${TESTK}" > gpurun_out/t_sub.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/t_sub.log | tail -60
tail -3 gpurun_out/t_sub.log
exit $rc
