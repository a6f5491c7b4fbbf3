set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in "NOALIAS=0 GTR_GRAPH_COLL=0" "NOALIAS=1 GTR_GRAPH_COLL=0" "NOALIAS=1 GTR_GRAPH_COLL=1"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 -X faulthandler -u scripts/dbg/twoclass_dbg.py 2>&1 | grep -v "amdgpu.ids" | tail -25
done
exit 0
