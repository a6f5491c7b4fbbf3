# round profile set: rocprofv3 kernel stats + PMC HBM traffic (separate passes) for C2,
# C3 and the B=8192 gather workload; then the default bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-v7}
# heartbeat: long PMC passes print nothing for minutes
(while true; do sleep 30; date >> gpurun_out/heartbeat.log; done) &
HB=$!
trap "kill $HB" EXIT
prof() {  # name, bench args
  local NAME=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$NAME -o run --output-format csv -- python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/prof_$NAME.json 2> gpurun_out/prof_$NAME.err || { tail -20 gpurun_out/prof_$NAME.err; exit 1; }
  cp gpurun_out/prof_$NAME/run_kernel_stats.csv gpurun_out/${NAME}_${V}_kernel_stats.csv
  rm -f gpurun_out/prof_$NAME/run_kernel_trace.csv  # large; the stats are what is kept
  echo "== $NAME"; python scripts/kstats.py gpurun_out/prof_$NAME/run_kernel_stats.csv
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${NAME}_$C -o run --output-format csv -- python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/pmc_${NAME}_$C.json 2> gpurun_out/pmc_${NAME}_$C.err || { tail -20 gpurun_out/pmc_${NAME}_$C.err; exit 1; }
  done
  python scripts/pmc_parse.py gpurun_out/pmc_${NAME}_FETCH_SIZE gpurun_out/pmc_${NAME}_WRITE_SIZE > gpurun_out/${NAME}_pmc.json
  rm -rf gpurun_out/pmc_${NAME}_FETCH_SIZE gpurun_out/pmc_${NAME}_WRITE_SIZE
  python -c "import json; d=json.load(open('gpurun_out/${NAME}_pmc.json')); print({k: round(v.get('hbm_bytes_per_launch', v.get('hbm_bytes_per_step', 0))) for k, v in d.items()})"
}
if [ -z "${ONLY_BIG:-}" ]; then
prof c2 --config c2 --steps 200 --warmup 20
prof c3 --config c3 --steps 200 --warmup 20
fi
prof c3_b8192 --config c3 --batch-size 8192 --num-batches 4 --steps 30 --warmup 5
if [ -n "${WITH_C5:-}" ]; then
prof c5 --config c5 --num-batches 4 --steps 30 --warmup 5
fi
