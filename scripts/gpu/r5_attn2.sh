set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TESTK="${TESTK:-split or long_sessions or edge_cases or halo or c4}" KB="c3:8192 c4:1024" bash scripts/gpu/r5_attn.sh || exit 1
