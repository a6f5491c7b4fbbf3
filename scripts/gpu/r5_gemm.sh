set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${TESTK:-split or ffn or c4 or long_sessions}" > gpurun_out/t_gemm.log 2>&1 || { tail -40 gpurun_out/t_gemm.log; exit 1; }
tail -2 gpurun_out/t_gemm.log
for v in base ${VARS:-NOMMA}; do
  L=$PWD/gat-recommendation_amd/build/libgtr_hip.so
  [ $v != base ] && L=$PWD/gat-recommendation_amd/build/var_$v/libgtr_hip.so
  for cb in "c3 8192" "c4 1024"; do
    echo "== $v $cb"
    GTR_SPLIT=1 GTR_LIB=$L timeout -k 10 200 python3 -u scripts/dbg/kbench.py $cb 2>&1 | grep "^{" || exit 1
  done
done
