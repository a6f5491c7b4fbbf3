#!/bin/bash
# Split-path checks: its GPU tests (and the SyncBN / multi-GPU ones), the DP-trainer
# diagnostic, then C3 at B = 8192 and C5 at B = 1024 with the split (default) and the fused
# (GTR_SPLIT=0) layer path, with rocprofv3 kernel stats of the split C3 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-split}
XFLAG= bash scripts/gpu/tests.sh "${2:-test_gpu_split or sync_bn or multigpu}" ${TAG}
rc=$?; [ $rc -le 1 ] || exit $rc
if [ "${DPDBG:-1}" = "1" ]; then
  timeout -k 10 500 python3 -u scripts/dbg/dp_trainer.py > gpurun_out/${TAG}_dp.log 2>&1 || { tail -5 gpurun_out/${TAG}_dp.log; exit 1; }
  grep ntrain gpurun_out/${TAG}_dp.log
fi
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --c1-reps 0 --tail-probe 0 --steps 30 --warmup 5"
for mode in 1 0; do
  GTR_SPLIT=$mode timeout -k 10 300 python3 bench.py --config c3 --batch-size 8192 $LEAN > gpurun_out/${TAG}_c3b8192_s$mode.json 2> gpurun_out/${TAG}_c3b8192_s$mode.err || { tail -20 gpurun_out/${TAG}_c3b8192_s$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_c3b8192_s$mode.json'));print('c3 b8192 split=$mode', d['value'], d['ms_per_step'])"
done
GTR_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 bench.py --config c3 --batch-size 8192 $LEAN > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
cp "$(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_c3b8192_kernel_stats.csv
rm -rf gpurun_out/prof_${TAG}
python3 scripts/kstats.py gpurun_out/${TAG}_c3b8192_kernel_stats.csv
for mode in 1 0; do
  GTR_SPLIT=$mode timeout -k 10 300 python3 bench.py --config c5 --batch-size 1024 $LEAN > gpurun_out/${TAG}_c5b1024_s$mode.json 2> gpurun_out/${TAG}_c5b1024_s$mode.err || { tail -20 gpurun_out/${TAG}_c5b1024_s$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_c5b1024_s$mode.json'));print('c5 b1024 split=$mode', d['value'], d['ms_per_step'])"
done
exit $rc
