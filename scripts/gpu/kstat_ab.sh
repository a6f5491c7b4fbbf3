#!/bin/bash
# rocprofv3 kernel stats of the lean C2 line under several environment settings.
# usage: scripts/gpu/kstat_ab.sh TAG "ENV1" "ENV2" ...   ("-": none)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
LEAN="--config ${CFG:-c2} --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --c1-reps 0 --tail-probe 0 --steps 200 --warmup 20 ${BARGS:-}"
i=0
for e in "$@"; do
  i=$((i+1))
  E=""; [ "$e" != "-" ] && E="$e"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$i -o run --output-format csv -- \
    python3 bench.py $LEAN > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  cp "$(find gpurun_out/prof_${TAG}_$i -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_${i}_kernel_stats.csv
  rm -rf gpurun_out/prof_${TAG}_$i
  echo "== [$e]"
  python3 scripts/kstats.py gpurun_out/${TAG}_${i}_kernel_stats.csv | head -8
done
