set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name args (env set by caller)
  local N=$1; shift
  timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 > gpurun_out/r1_$N.json 2> gpurun_out/r1_$N.err || { tail -30 gpurun_out/r1_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r1_$N.json')); c=d['config']; print('$N', d['value'], d['ms_per_step'], c['final_loss'], c['transport'], c['lagged_sweep'])"
}
run gloo_free_dp_eager --dp --lagged 0
export GTR_FORCE_PG=1
GTR_GRAPH_COLL=0 run rccl_dp_eager_split --dp --lagged 0
GTR_GRAPH_COLL=0 run rccl_dp_lagged_split --dp --lagged 1
GTR_GRAPH_COLL=1 run rccl_dp_eager_graph --dp --lagged 0
GTR_GRAPH_COLL=1 run rccl_dp_lagged_graph --dp --lagged 1
GTR_GRAPH_COLL=1 run rccl_c3_dp_lagged_graph --config c3 --dp --lagged 1
GTR_GRAPH_COLL=1 run rccl_c2_syncbn_graph --sync-bn --lagged 1
GTR_GRAPH_COLL=0 run rccl_c2_syncbn_split --sync-bn --lagged 1
