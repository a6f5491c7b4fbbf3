set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
GTR_LIB=$PWD/gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 200 python3 -u scripts/phase_timing.py --steps 40 2>&1 | grep -v amdgpu.ids
