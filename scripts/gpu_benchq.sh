# default bench line (C2 + CPU baseline + gather + Recall@10 legs) and C3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -30 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 600 python bench.py --config c3 --cpu-seconds 10 --gather-batch 0 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
