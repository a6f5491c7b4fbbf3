# parity tests, then smoke + bench + rocprof kernel stats (CFG=c2|c3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c2}
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=8 > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
bash scripts/gpu_bench.sh
