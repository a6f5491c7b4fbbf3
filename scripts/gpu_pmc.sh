# PMC HBM-traffic passes (one counter per pass, kernel trace only) for the step-tail and layer kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c2}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${CFG}_$C -o run --output-format csv -- python bench.py --config $CFG --steps 50 --warmup 10 --cpu-seconds 0 > gpurun_out/pmc_${CFG}_$C.json 2> gpurun_out/pmc_${CFG}_$C.err || { tail -30 gpurun_out/pmc_${CFG}_$C.err; exit 1; }
done
python scripts/pmc_parse.py gpurun_out/pmc_${CFG}_FETCH_SIZE gpurun_out/pmc_${CFG}_WRITE_SIZE > gpurun_out/pmc_${CFG}.json
cat gpurun_out/pmc_${CFG}.json
