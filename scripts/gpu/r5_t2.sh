set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "${TESTK}" > gpurun_out/t_sub.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/t_sub.log | tail -20
tail -2 gpurun_out/t_sub.log
[ $rc -eq 0 ] || exit $rc
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps 500 --warmup 20"
for r in 1 2; do
  for v in 1 0; do
    GTR_FORCE_PG=1 GTR_DP_NOALIAS=$v timeout -k 10 300 python3 bench.py --dp $L 2> gpurun_out/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c2 dp world1 NOALIAS=$v', d['ms_per_step'])" || { tail -20 gpurun_out/ab.err; exit 1; }
  done
  timeout -k 10 300 python3 bench.py --config c4 --global-batch 1024 $L 2> gpurun_out/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c4 1024', d['ms_per_step'])" || { tail -20 gpurun_out/ab.err; exit 1; }
done
