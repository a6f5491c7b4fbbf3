set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in "GTR_SPLIT=1" "GTR_SPLIT=1 GTR_GEMM_GEN=1"; do
  for cb in "c3 8192" "c3 1024"; do
    echo "== $v $cb"
    env $v timeout -k 10 200 python3 -u scripts/dbg/kbench.py $cb 2>&1 | grep "^{" || exit 1
  done
done
