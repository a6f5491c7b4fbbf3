set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TESTK="split or long_sessions or edge_cases" KB="c3:8192 c4:1024" bash scripts/gpu/r5_attn.sh || exit 1
bash scripts/gpu/phases.sh "c4:1024" > gpurun_out/ph2.log 2>&1 || { tail -20 gpurun_out/ph2.log; exit 1; }
head -16 gpurun_out/ph2.log
