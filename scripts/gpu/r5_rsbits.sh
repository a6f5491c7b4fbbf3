set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sort or parity or fullsize or c4 or sharded or split" > gpurun_out/t_rs.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/t_rs.log | tail -20
tail -2 gpurun_out/t_rs.log
[ $rc -eq 0 ] || exit $rc
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps 200 --warmup 20"
for r in 1 2; do
  for c in "c3 --batch-size 8192" "c4 --global-batch 1024"; do
    for b in 10 9; do
      GTR_RS_BITS=$b timeout -k 10 300 python3 bench.py --config $c $L 2> gpurun_out/rs.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$c', 'bits $b', d['ms_per_step'])" || { tail -20 gpurun_out/rs.err; exit 1; }
    done
  done
done
