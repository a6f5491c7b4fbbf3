set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gap
export TMPDIR=/tmp
run() {  # name args
  local N=$1; shift
  timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/gap/$N.json 2> gpurun_out/gap/$N.err || { tail -20 gpurun_out/gap/$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/gap/$N.json')); print('$N', d['value'], d['ms_per_step'])"
}
run graph
run nograph --no-graph
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/tr_graph -o run -- python3 bench.py --steps 50 --warmup 10 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > /dev/null 2> gpurun_out/gap/trg.err || { tail -20 gpurun_out/gap/trg.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/tr_nograph -o run -- python3 bench.py --no-graph --steps 50 --warmup 10 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > /dev/null 2> gpurun_out/gap/trn.err || { tail -20 gpurun_out/gap/trn.err; exit 1; }
find gpurun_out/gap -name "*.csv" | head
