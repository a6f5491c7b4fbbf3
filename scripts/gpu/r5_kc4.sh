set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp ROUND=r05 PMC=0
GTR_SPLIT=1 bash scripts/gpu/profile.sh c4 c4_b1024 --global-batch 1024 > gpurun_out/p_c4.log 2>&1 || { tail -20 gpurun_out/p_c4.log; exit 1; }
python3 scripts/kstat_summary.py gpurun_out/c4_b1024_kernel_stats.csv 24
python3 -c "import json; d=json.loads(open('gpurun_out/c4_b1024_bench.json').read().strip().splitlines()[-1]); print('c4', d['ms_per_step'])"
