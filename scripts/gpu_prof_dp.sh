set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pdp
export TMPDIR=/tmp
export GTR_FORCE_PG=1 GTR_GRAPH_COLL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pdp/dp -o run -- python3 bench.py --dp --lagged 1 --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/pdp/dp.json 2> gpurun_out/pdp/dp.err || { tail -20 gpurun_out/pdp/dp.err; exit 1; }
unset GTR_FORCE_PG GTR_GRAPH_COLL
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pdp/lag -o run -- python3 bench.py --lagged 1 --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/pdp/lag.json 2> gpurun_out/pdp/lag.err || { tail -20 gpurun_out/pdp/lag.err; exit 1; }
find gpurun_out/pdp -name "*kernel_stats.csv" | head
