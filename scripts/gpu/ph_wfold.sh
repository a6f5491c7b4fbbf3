set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for W in 1 0; do
  GTR_WFOLD=$W GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --config c2 --steps 30 > gpurun_out/ph_w$W.txt 2> gpurun_out/ph_w$W.err || { tail -20 gpurun_out/ph_w$W.err; exit 1; }
  echo "== WFOLD=$W"; cat gpurun_out/ph_w$W.txt
done
