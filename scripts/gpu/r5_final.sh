# Round-5 final measurements on the final tree: profiles (stats + PMC + bench line) per
# configuration, then the default bench line exactly as the driver runs it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp ROUND=r05
mkdir -p gpurun_out
for spec in "c2:c2:" "c3:c3_b8192:--batch-size=8192" "c4:c4_b1024:--global-batch=1024" "c5:c5_b1024:--batch-size=1024" "c5:c5_b8192:--batch-size=8192"; do
  IFS=: read -r cfg tag extra <<< "$spec"
  echo "== $tag"
  bash scripts/gpu/profile.sh $cfg $tag $extra > gpurun_out/p_$tag.log 2>&1 || { tail -20 gpurun_out/p_$tag.log; exit 1; }
  grep "pmc per step" gpurun_out/p_$tag.log
done
echo "== c4_b1024_split"
GTR_SPLIT=1 bash scripts/gpu/profile.sh c4 c4_b1024_split --global-batch=1024 > gpurun_out/p_c4s.log 2>&1 || { tail -20 gpurun_out/p_c4s.log; exit 1; }
echo "== default bench"
timeout -k 10 900 python3 bench.py > gpurun_out/default_bench.json 2> gpurun_out/default_bench.err || { tail -30 gpurun_out/default_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/default_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'), d.get('trainer_epoch',{}).get('ms_per_step'), [ (l.get('global_batch'), l.get('value'), l.get('ms_per_step')) for l in d.get('strong_scaling',{}).get('legs',[])])"
