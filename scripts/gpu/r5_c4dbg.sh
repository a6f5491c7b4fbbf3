set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in rows new; do
  GTR_ATTN=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_c4.py -m gpu -x -s -q --timeout 280 --timeout-method thread -p no:cacheprovider -k "bitwise_dp and 2" > gpurun_out/c4dbg_$v.log 2>&1
  echo "== $v rc=$?"; grep -E "^step|passed|failed" gpurun_out/c4dbg_$v.log
done
