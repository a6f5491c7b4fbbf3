set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu/r5_gph.sh || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "split or ffn" > gpurun_out/t_split.log 2>&1 || { tail -30 gpurun_out/t_split.log; exit 1; }
tail -2 gpurun_out/t_split.log
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0 --steps 200 --warmup 20"
for c in "c3 --batch-size 8192" "c5 --batch-size 8192" "c4 --global-batch 1024"; do
  timeout -k 10 300 python3 bench.py --config $c $L 2> gpurun_out/g2.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['value'])" || { tail -20 gpurun_out/g2.err; exit 1; }
done
