set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "split or parity or fullsize or pipeline" > gpurun_out/t_ct.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/t_ct.log | tail -20
tail -2 gpurun_out/t_ct.log
[ $rc -eq 0 ] || exit $rc
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps 2000 --warmup 50"
for r in 1 2 3; do
  for lib in build/convt0 build; do
    GTR_LIB=$PWD/gat-recommendation_amd/$lib/libgtr_hip.so timeout -k 10 300 python3 bench.py $L 2> gpurun_out/ct.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c2', '$lib', d['ms_per_step'])" || { tail -20 gpurun_out/ct.err; exit 1; }
  done
done
for lib in build/convt0 build; do
  GTR_LIB=$PWD/gat-recommendation_amd/$lib/libgtr_hip.so timeout -k 10 300 python3 bench.py --config c3 ${L/2000/1000} 2> gpurun_out/ct.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c3', '$lib', d['ms_per_step'])" || { tail -20 gpurun_out/ct.err; exit 1; }
done
