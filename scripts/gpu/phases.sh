set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --steps 30 > gpurun_out/phases_c2.txt 2>gpurun_out/phases_c2.err
cat gpurun_out/phases_c2.txt
