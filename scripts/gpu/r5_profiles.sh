# Round-5 profiles: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes + bench line
# per configuration (scripts/gpu/profile.sh), copied under profiles/r05 by the caller.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp ROUND=r05
for spec in ${SPECS:-"c2:c2:" "c3:c3_b8192:--batch-size 8192" "c4:c4_b1024:--global-batch 1024"}; do
  IFS=: read -r cfg tag extra <<< "$spec"
  echo "== $tag"
  bash scripts/gpu/profile.sh $cfg $tag $extra > gpurun_out/p_$tag.log 2>&1 || { tail -20 gpurun_out/p_$tag.log; exit 1; }
  grep "pmc per step" gpurun_out/p_$tag.log
  python3 scripts/kstat_summary.py gpurun_out/${tag}_kernel_stats.csv 8
done
