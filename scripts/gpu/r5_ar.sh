set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps 200 --warmup 20"
for r in 1 2; do
  for c in "c3 --batch-size 8192" "c4 --global-batch 1024"; do
    for lib in ${BASE:-build} ${VARIANT:-build/ar512}; do
      GTR_SPLIT=1 GTR_LIB=$PWD/gat-recommendation_amd/$lib/libgtr_hip.so timeout -k 10 300 python3 bench.py --config $c $L 2> gpurun_out/ar.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$c', '$lib', d['ms_per_step'])" || { tail -20 gpurun_out/ar.err; exit 1; }
    done
  done
done
