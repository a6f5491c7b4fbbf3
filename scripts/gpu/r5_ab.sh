# A/B of an env toggle on the bench step (same box, alternating).  usage: AB_VAR=NAME AB_A=x AB_B=y CFGS="..." r5_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps ${STEPS:-300} --warmup 20"
IFS=';' read -ra CS <<< "${CFGS:-c3 --batch-size 8192;c4 --global-batch 1024}"
for r in 1 2; do
  for c in "${CS[@]}"; do
    for v in "$AB_A" "$AB_B"; do
      env $AB_VAR=$v timeout -k 10 300 python3 bench.py --config $c $L 2> gpurun_out/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$c', '$AB_VAR=$v', d['ms_per_step'])" || { tail -20 gpurun_out/ab.err; exit 1; }
    done
  done
done
