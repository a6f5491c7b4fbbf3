#!/bin/bash
# The multi-GPU bench tests (shared-device gloo rehearsals, strong legs) and the default
# bench line (N = 1, every leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multigpu.py -m gpu -x -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider -k "bench" > gpurun_out/t_bench.log 2>&1 || { tail -40 gpurun_out/t_bench.log; exit 1; }
tail -3 gpurun_out/t_bench.log
timeout -k 10 900 python3 bench.py > gpurun_out/default_bench.json 2> gpurun_out/default_bench.err \
  || { tail -30 gpurun_out/default_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/default_bench.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['strong_scaling'],indent=1))"
