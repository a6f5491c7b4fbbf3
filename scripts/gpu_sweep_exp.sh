# chain-sweep experiments: blocks per launch and slot weights (C2), step time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  timeout -k 10 120 python bench.py --config ${CFG:-c2} --steps 300 --warmup 30 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 > gpurun_out/x.json 2> gpurun_out/x.err || { tail -20 gpurun_out/x.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/x.json')); print('$1', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
GTR_CHAIN_SWEEP=0 run off
for B in 32 64 128 240; do GTR_SWEEP_BLOCKS=$B run blocks=$B; done
GTR_SWEEP_WTS=1,1,0,1,1 run w11011
GTR_SWEEP_WTS=0,1,1,1,0 run w01110
GTR_SWEEP_WTS=1,0,0,0,0 run w10000
GTR_SWEEP_WTS=0,0,0,0,1 run w00001
GTR_SWEEP_WTS=0,0,1,0,0 run w00100
CFG=c3 GTR_CHAIN_SWEEP=0 run c3off
CFG=c3 run c3on
for B in 64 128; do CFG=c3 GTR_SWEEP_BLOCKS=$B run c3blocks=$B; done
