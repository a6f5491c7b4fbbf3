# round-end artifacts: default bench lines + kernel stats + PMC traffic (C2, C3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-v10}
(while true; do sleep 30; date >> gpurun_out/heartbeat.log; done) &
HB=$!
trap "kill $HB" EXIT
for CFG in c2 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/prof_$CFG.json 2> gpurun_out/prof_$CFG.err || { tail -20 gpurun_out/prof_$CFG.err; exit 1; }
cp gpurun_out/prof_$CFG/run_kernel_stats.csv gpurun_out/${CFG}_${V}_kernel_stats.csv
rm -rf gpurun_out/prof_$CFG
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${CFG}_$C -o run --output-format csv -- python bench.py --config $CFG --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/pmc_${CFG}_$C.json 2> gpurun_out/pmc_${CFG}_$C.err || { tail -20 gpurun_out/pmc_${CFG}_$C.err; exit 1; }
done
python scripts/pmc_parse.py gpurun_out/pmc_${CFG}_FETCH_SIZE gpurun_out/pmc_${CFG}_WRITE_SIZE > gpurun_out/${CFG}_pmc.json
rm -rf gpurun_out/pmc_${CFG}_FETCH_SIZE gpurun_out/pmc_${CFG}_WRITE_SIZE
cp gpurun_out/${CFG}_pmc.json profiles/r01/${CFG}_pmc.json
done
timeout -k 10 600 python bench.py > gpurun_out/c2_${V}_bench.json 2> gpurun_out/c2_${V}_bench.err || { tail -30 gpurun_out/c2_${V}_bench.err; exit 1; }
timeout -k 10 600 python bench.py --config c3 > gpurun_out/c3_${V}_bench.json 2> gpurun_out/c3_${V}_bench.err || { tail -30 gpurun_out/c3_${V}_bench.err; exit 1; }
timeout -k 10 600 python bench.py --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/c3_b8192_${V}_bench.json 2> gpurun_out/c3_b8192_${V}_bench.err || { tail -30 gpurun_out/c3_b8192_${V}_bench.err; exit 1; }
timeout -k 10 600 python bench.py --config c5 --num-batches 8 --steps 50 --warmup 10 --recall-steps 0 --e2e-steps 0 --gather-batch 0 --cpu-seconds 0 > gpurun_out/c5_${V}_bench.json 2> gpurun_out/c5_${V}_bench.err || { tail -30 gpurun_out/c5_${V}_bench.err; exit 1; }
for n in c2 c3 c3_b8192 c5; do python -c "import json; d=json.load(open('gpurun_out/${n}_${V}_bench.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"; done
