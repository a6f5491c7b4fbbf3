set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for cb in "c3 1024" "c3 8192"; do
  GTR_SPLIT=1 GTR_LIB=$PWD/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 200 python3 -u scripts/dbg/gemm_phases.py $cb 2>&1 | grep -v amdgpu.ids || exit 1
done
