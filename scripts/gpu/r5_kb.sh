set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
[ -n "$TESTK" ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "$TESTK" > gpurun_out/t_kb.log 2>&1 || { tail -40 gpurun_out/t_kb.log; exit 1; }; tail -2 gpurun_out/t_kb.log; }
for v in ${VARIANTS:-"GTR_SPLIT=1"}; do
  for cb in ${CBS:-"c3:8192 c3:1024"}; do
    echo "== $v $cb"
    env ${v//,/ } timeout -k 10 200 python3 -u scripts/dbg/kbench.py ${cb%%:*} ${cb##*:} 2>&1 | grep "^{" || exit 1
  done
done
