# Round-5 one-GPU numbers: DP C2 over a one-rank RCCL group (aliased vs real collective
# captured), the sharded c4 steps (fitted vs static blocks), two alternating passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --c1-reps 0 --tail-probe 0 --strong-batches 0"
one() { local tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/n_$tag.json 2> gpurun_out/n_$tag.err || { tail -20 gpurun_out/n_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/n_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['value'], d['config'].get('step_graph'))"; }
for r in 1 2; do
  GTR_FORCE_PG=1 one dp_alias python3 bench.py --dp --steps 500 --warmup 20 $L
  GTR_FORCE_PG=1 GTR_DP_NOALIAS=1 GTR_GRAPH_COLL=1 one dp_rccl python3 bench.py --dp --steps 500 --warmup 20 $L
  one c4_1024 python3 bench.py --config c4 --global-batch 1024 --steps 200 --warmup 20 $L
  one c4_1024_static python3 bench.py --config c4 --global-batch 1024 --fit-blocks 0 --steps 200 --warmup 20 $L
  GTR_SPLIT=1 one c4_1024_split python3 bench.py --config c4 --global-batch 1024 --steps 200 --warmup 20 $L
done
one c4_8192 python3 bench.py --config c4 --steps 50 --warmup 10 $L
one c4_65536 python3 bench.py --config c4 --global-batch 65536 --steps 10 --warmup 3 $L
one c3_65536 python3 bench.py --config c3 --batch-size 65536 --steps 10 --warmup 3 $L
