set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-v8}
(while true; do sleep 30; date >> gpurun_out/heartbeat.log; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --config c2 --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/prof_c2.json 2> gpurun_out/prof_c2.err || { tail -20 gpurun_out/prof_c2.err; exit 1; }
cp gpurun_out/prof_c2/run_kernel_stats.csv gpurun_out/c2_${V}_kernel_stats.csv
rm -f gpurun_out/prof_c2/run_kernel_trace.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_c2_$C -o run --output-format csv -- python bench.py --config c2 --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/pmc_c2_$C.json 2> gpurun_out/pmc_c2_$C.err || { tail -20 gpurun_out/pmc_c2_$C.err; exit 1; }
done
python scripts/pmc_parse.py gpurun_out/pmc_c2_FETCH_SIZE gpurun_out/pmc_c2_WRITE_SIZE > gpurun_out/c2_pmc.json
rm -rf gpurun_out/pmc_c2_FETCH_SIZE gpurun_out/pmc_c2_WRITE_SIZE
cp gpurun_out/c2_pmc.json profiles/r01/c2_pmc.json
timeout -k 10 600 python bench.py > gpurun_out/c2_${V}_bench.json 2> gpurun_out/c2_${V}_bench.err || { tail -30 gpurun_out/c2_${V}_bench.err; exit 1; }
cat gpurun_out/c2_${V}_bench.json
