#!/bin/bash
# Full GPU parity suite, then the lean C2 bench line (no CPU / recall / e2e legs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
XFLAG= bash scripts/gpu/tests.sh "${1:-}" ${2:-check} || exit 1
LEAN="--config c2 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --steps 400 --warmup 30"
timeout -k 10 300 python3 bench.py $LEAN > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err || { tail -20 gpurun_out/check_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/check_bench.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['tail_kernel'])"
